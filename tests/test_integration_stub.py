"""Boundary drift guard: the Rust `extern "C"` binding that INTEGRATION.md gives a maintainer of the
reference (src/model/scene.rs:35-57 calls render_diff; src/bin/train.rs:182 the training step)
must declare every entry point of include/raymarch.h and include/rm_host.h with the same
parameters in the same order (types mapped C -> Rust), and every `#[repr(C)]` struct of the
headers with the same fields in the same order. The stub is documentation (no Rust toolchain in
this image), so this CPU test is what keeps it from drifting when a signature changes."""
import os
import re

import pytest

from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in ("raymarch.h", "rm_host.h")]
DOC = os.path.join(ROOT, "INTEGRATION.md")

BASE = {"float": "f32", "double": "f64", "int32_t": "i32", "int64_t": "i64", "uint64_t": "u64", "uint32_t": "u32",
        "uint16_t": "u16", "uint8_t": "u8", "int": "c_int", "char": "c_char", "void": "c_void"}


def _strip_c_comments(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", " ", text)


def _c_type(decl, is_param=True, field=False):
    """Normalise one C declaration ('const float* eye', 'float eye[3]', 'rm_context** out') to
    the Rust spelling of its type ('*const f32', '*mut f32', '*mut *mut rm_context')."""
    decl = " ".join(decl.replace("*", " * ").split())
    array = re.search(r"\[([^\]]*)\]\s*$", decl)
    if array:
        decl = decl[:array.start()].strip()
    toks = decl.split()
    if (is_param or field) and len(toks) > 1 and re.match(r"^[A-Za-z_]\w*$", toks[-1]) and toks[-1] not in BASE:
        toks = toks[:-1]  # the parameter / field name
    const = "const" in toks
    toks = [t for t in toks if t != "const"]
    stars = toks.count("*")
    base = [t for t in toks if t != "*"]
    assert len(base) == 1, decl
    name = BASE.get(base[0], base[0])
    if array and not field:  # an array parameter is a pointer
        return ("*const " if const else "*mut ") + name
    if array:
        return f"[{name}; {array.group(1).strip()}]"
    if stars == 0:
        return name
    # the pointee's const applies to the innermost level (`const T**` = pointer to pointer to const T)
    out = ("*const " if const else "*mut ") + name
    for _ in range(stars - 1):
        out = "*mut " + out
    return out


def _split_top(s):
    parts, depth, cur = [], 0, ""
    for i, ch in enumerate(s):
        if ch in "([<":
            depth += 1
        elif ch in ")]>" and not (ch == ">" and i > 0 and s[i - 1] == "-"):  # not the `->` of a fn type
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    return [p.strip() for p in parts if p.strip()]


def _c_fnptr(field):
    """'int (*all_reduce_sum)(void* state, float* buf)' -> ('all_reduce_sum', 'fn(*mut c_void,*mut f32)->c_int')."""
    m = re.match(r"^(.*?)\(\s*\*\s*(\w+)\s*\)\s*\((.*)\)$", field.strip(), flags=re.S)
    ret = _c_type(m.group(1), is_param=False)
    args = [] if m.group(3).strip() in ("", "void") else [_c_type(a) for a in _split_top(m.group(3))]
    return m.group(2), "fn(" + ",".join(args) + ")" + ("" if ret == "c_void" else "->" + ret)


def header_api():
    fns, structs = {}, {}
    for h in HEADERS:
        text = _strip_c_comments(open(h).read())
        text = re.sub(r"#[^\n]*", " ", text)
        for m in re.finditer(r"typedef\s+struct\s+(\w+)\s*\{(.*?)\}\s*\w+\s*;", text, flags=re.S):
            fields = []
            for f in [x.strip() for x in m.group(2).split(";") if x.strip()]:
                if "(*" in f.replace(" ", ""):
                    fields.append(_c_fnptr(f))
                    continue
                # `int32_t width, height` declares two fields of one type
                first, *more = [x.strip() for x in f.split(",")]
                t = _c_type(first, is_param=False, field=True)
                fields.append((re.findall(r"(\w+)\s*(?:\[[^\]]*\])?\s*$", first)[0], t))
                for name in more:
                    fields.append((name, t))
            structs[m.group(1)] = fields
        text = re.sub(r"typedef\s+struct\s+\w+\s*\{.*?\}\s*\w+\s*;", " ", text, flags=re.S)
        for m in re.finditer(r"([\w\s\*]+?)\b(rmh?_\w+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
            ret = _c_type(m.group(1).replace("extern", ""), is_param=False)
            args = [] if m.group(3).strip() in ("", "void") else [_c_type(a) for a in _split_top(m.group(3))]
            fns[m.group(2)] = (args, ret)
    return fns, structs


def _rust_type(t):
    t = " ".join(t.split())
    t = re.sub(r"^Option<(.*)>$", r"\1", t)
    if "fn(" in t:  # fn pointer: drop unsafe / extern "C" / parameter names
        m = re.match(r'^(?:unsafe\s+)?(?:extern\s+"C"\s+)?fn\s*\((.*)\)\s*(?:->\s*(.+))?$', t)
        args = [_rust_type(a.split(":", 1)[1] if re.match(r"^\w+\s*:", a) else a) for a in _split_top(m.group(1))]
        return "fn(" + ",".join(args) + ")" + (("->" + _rust_type(m.group(2))) if m.group(2) else "")
    return t


def doc_api():
    fns, structs = {}, {}
    blocks = re.findall(r"```rust\n(.*?)```", open(DOC).read(), flags=re.S)
    for b in blocks:
        b = re.sub(r"//[^\n]*", " ", b)
        b = re.sub(r"/\*.*?\*/", " ", b, flags=re.S)
        for m in re.finditer(r"pub\s+fn\s+(rmh?_\w+)\s*\((.*?)\)\s*(?:->\s*([^;{]+?))?\s*;", b, flags=re.S):
            args = [_rust_type(a.split(":", 1)[1]) for a in _split_top(m.group(2))]
            assert m.group(1) not in fns, f"{m.group(1)} declared twice in INTEGRATION.md"
            fns[m.group(1)] = (args, _rust_type(m.group(3)) if m.group(3) else "c_void")
        for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive\([^)]*\)\]\s*)?pub\s+struct\s+(\w+)\s*\{(.*?)\}\s*(?=#|pub|extern|$|\n)",
                             b, flags=re.S):
            body = m.group(2)
            if "_p:" in body:  # opaque handle
                continue
            fields = []
            for f in _split_top(body):
                name, t = f.split(":", 1)
                fields.append((name.replace("pub", "").strip(), _rust_type(t)))
            structs[m.group(1)] = fields
    return fns, structs


def test_header_parser_sanity():
    fns, structs = header_api()
    assert fns["rm_create"] == (["i32", "*mut c_void", "*mut *mut rm_context"], "c_int")
    assert fns["rmh_camera_rays"][0][2] == "*const f32" and fns["rmh_last_error"] == ([], "*const c_char")
    assert ("all_reduce_sum", "fn(*mut c_void,*mut f32,i64,*mut c_void)->c_int") in structs["rmh_collective"]
    assert ("height", "i32") in structs["rmh_train_config"] and ("file", "[c_char; RMH_PATH_MAX]") in \
        structs["rmh_camera_entry"]
    assert len(fns) > 60


def test_rust_stub_declares_every_entry_point():
    hf, _ = header_api()
    df, _ = doc_api()
    missing = sorted(set(hf) - set(df))
    extra = sorted(set(df) - set(hf))
    assert not missing, f"INTEGRATION.md lacks {missing}"
    assert not extra, f"INTEGRATION.md declares functions the headers do not: {extra}"


@pytest.mark.parametrize("name", sorted(header_api()[0]))
def test_rust_signature_matches_header(name):
    hargs, hret = header_api()[0][name]
    dargs, dret = doc_api()[0][name]
    assert len(dargs) == len(hargs), (name, "parameter count", dargs, hargs)
    for i, (d, h) in enumerate(zip(dargs, hargs)):
        assert d == h, (name, f"parameter {i}", d, h)
    assert dret == hret, (name, "return", dret, hret)


def test_rust_structs_match_header():
    _, hs = header_api()
    _, ds = doc_api()
    assert set(hs) <= set(ds), sorted(set(hs) - set(ds))
    for name, fields in hs.items():
        assert ds[name] == fields, (name, ds[name], fields)
