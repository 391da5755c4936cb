// librm_host.so, part 1: files. PNG codec over zlib (util.rs:4-33 uses the `image` crate),
// a small JSON reader/writer for cameras.json (train.rs:15-21, generate.rs:13-18) and
// scene.json (train.rs:238-262), with serde_json's pretty layout and ryu float formatting.
#include <sys/stat.h>
#include <zlib.h>

#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "rmh_common.hpp"

namespace rmh {

static thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

bool read_file(const std::string& path, std::string& out) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  out.clear();
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
  const bool ok = !std::ferror(f);
  std::fclose(f);
  return ok;
}

bool write_file(const std::string& path, const std::string& data) {
  if (!make_parent_dirs(path)) return false;
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  const bool ok = std::fwrite(data.data(), 1, data.size(), f) == data.size();
  return (std::fclose(f) == 0) && ok;
}

bool make_dirs(const std::string& dir) {
  if (dir.empty()) return true;
  std::string cur;
  for (size_t i = 0; i <= dir.size(); ++i) {
    if (i == dir.size() || dir[i] == '/') {
      if (!cur.empty() && cur != "/" && mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
    if (i < dir.size()) cur.push_back(dir[i]);
  }
  return true;
}

std::string dirname_of(const std::string& path) {
  const size_t p = path.rfind('/');
  return p == std::string::npos ? std::string() : path.substr(0, p);
}

bool make_parent_dirs(const std::string& path) { return make_dirs(dirname_of(path)); }

std::string join_path(const std::string& dir, const std::string& name) {
  if (dir.empty() || (!name.empty() && name[0] == '/')) return name;
  return dir.back() == '/' ? dir + name : dir + "/" + name;
}

float sigmoid_f32(float x) { return 1.0f / (1.0f + std::exp(-x)); }
float softplus_f32(float x) { return std::log(1.0f + std::exp(x)); }

// ---- JSON -------------------------------------------------------------------------------

const Json* Json::get(const std::string& key) const {
  if (kind != Object) return nullptr;
  for (const auto& kv : obj)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

namespace {

struct Parser {
  const std::string& s;
  size_t i = 0;
  std::string err;

  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  bool bad(const char* what) {
    if (err.empty()) err = std::string(what) + " at offset " + std::to_string(i);
    return false;
  }
  bool lit(const char* w) {
    const size_t n = std::strlen(w);
    if (s.compare(i, n, w) != 0) return bad("invalid literal");
    i += n;
    return true;
  }
  static void utf8(std::string& o, unsigned cp) {
    if (cp < 0x80) {
      o.push_back((char)cp);
    } else if (cp < 0x800) {
      o.push_back((char)(0xC0 | (cp >> 6)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      o.push_back((char)(0xE0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  bool string(std::string& o) {
    if (s[i] != '"') return bad("expected string");
    ++i;
    while (i < s.size() && s[i] != '"') {
      char c = s[i++];
      if (c != '\\') {
        o.push_back(c);
        continue;
      }
      if (i >= s.size()) return bad("bad escape");
      c = s[i++];
      switch (c) {
        case '"': o.push_back('"'); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case 'u': {
          if (i + 4 > s.size()) return bad("bad \\u escape");
          unsigned cp = (unsigned)std::strtoul(s.substr(i, 4).c_str(), nullptr, 16);
          i += 4;
          utf8(o, cp);
          break;
        }
        default: return bad("bad escape");
      }
    }
    if (i >= s.size()) return bad("unterminated string");
    ++i;
    return true;
  }
  bool value(Json& v, int depth) {
    if (depth > 64) return bad("nesting too deep");
    ws();
    if (i >= s.size()) return bad("unexpected end");
    const char c = s[i];
    if (c == '{') {
      v.kind = Json::Object;
      ++i;
      ws();
      if (i < s.size() && s[i] == '}') {
        ++i;
        return true;
      }
      for (;;) {
        ws();
        std::string key;
        if (i >= s.size() || !string(key)) return bad("expected key");
        ws();
        if (i >= s.size() || s[i] != ':') return bad("expected ':'");
        ++i;
        Json child;
        if (!value(child, depth + 1)) return false;
        v.obj.emplace_back(std::move(key), std::move(child));
        ws();
        if (i < s.size() && s[i] == ',') {
          ++i;
          continue;
        }
        if (i < s.size() && s[i] == '}') {
          ++i;
          return true;
        }
        return bad("expected ',' or '}'");
      }
    }
    if (c == '[') {
      v.kind = Json::Array;
      ++i;
      ws();
      if (i < s.size() && s[i] == ']') {
        ++i;
        return true;
      }
      for (;;) {
        Json child;
        if (!value(child, depth + 1)) return false;
        v.arr.push_back(std::move(child));
        ws();
        if (i < s.size() && s[i] == ',') {
          ++i;
          continue;
        }
        if (i < s.size() && s[i] == ']') {
          ++i;
          return true;
        }
        return bad("expected ',' or ']'");
      }
    }
    if (c == '"') {
      v.kind = Json::String;
      return string(v.str);
    }
    if (c == 't') {
      v.kind = Json::Bool;
      v.b = true;
      return lit("true");
    }
    if (c == 'f') {
      v.kind = Json::Bool;
      return lit("false");
    }
    if (c == 'n') {
      v.kind = Json::Null;
      return lit("null");
    }
    // number
    const char* begin = s.c_str() + i;
    char* end = nullptr;
    v.num = std::strtod(begin, &end);
    if (end == begin) return bad("invalid value");
    v.kind = Json::Number;
    i += (size_t)(end - begin);
    return true;
  }
};

}  // namespace

bool json_parse(const std::string& text, Json& out, std::string& err) {
  Parser p{text};
  out = Json();
  if (!p.value(out, 0)) {
    err = p.err;
    return false;
  }
  p.ws();
  if (p.i != text.size()) {
    err = "trailing characters at offset " + std::to_string(p.i);
    return false;
  }
  return true;
}

// ryu's f32 "pretty" layout (the format serde_json writes): shortest round-trip digits d
// (length n) with decimal exponent so that value = 0.d * 10^kk.
std::string fmt_f32(float x) {
  if (!std::isfinite(x)) return "null";
  if (x == 0.0f) return std::signbit(x) ? "-0.0" : "0.0";
  char buf[64];
  const auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
  std::string sci(buf, r.ptr);  // [-]d[.ddd]e[+-]XX
  std::string out;
  size_t p = 0;
  if (sci[0] == '-') {
    out.push_back('-');
    p = 1;
  }
  const size_t e = sci.find('e');
  std::string digits;
  for (size_t k = p; k < e; ++k)
    if (sci[k] != '.') digits.push_back(sci[k]);
  const int exp10 = std::atoi(sci.c_str() + e + 1);
  const int n = (int)digits.size();
  const int kk = exp10 + 1;  // position of the decimal point
  const int k = kk - n;
  if (k >= 0 && kk <= 13) {
    out += digits + std::string((size_t)k, '0') + ".0";
  } else if (kk > 0 && kk <= 13) {
    out += digits.substr(0, (size_t)kk) + "." + digits.substr((size_t)kk);
  } else if (kk > -6 && kk <= 0) {
    out += "0." + std::string((size_t)(-kk), '0') + digits;
  } else if (n == 1) {
    out += digits + "e" + std::to_string(kk - 1);
  } else {
    out += digits.substr(0, 1) + "." + digits.substr(1) + "e" + std::to_string(kk - 1);
  }
  return out;
}

namespace {

void put_f32_array(std::string& o, const char* key, const float* v, size_t n, bool last) {
  o += "  \"";
  o += key;
  o += "\": [";
  if (n == 0) {
    o += "]";
  } else {
    for (size_t i = 0; i < n; ++i) {
      o += i ? ",\n    " : "\n    ";
      o += fmt_f32(v[i]);
    }
    o += "\n  ]";
  }
  o += last ? "\n" : ",\n";
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      case '\r': o += "\\r"; break;
      default:
        if ((unsigned char)c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", (unsigned char)c);
          o += b;
        } else {
          o.push_back(c);
        }
    }
  }
  return o;
}

bool num_array(const Json* v, std::vector<float>& out) {
  if (!v || v->kind != Json::Array) return false;
  out.clear();
  for (const auto& e : v->arr) {
    if (e.kind != Json::Number) return false;
    out.push_back((float)e.num);
  }
  return true;
}

// ---- PNG ----------------------------------------------------------------------------------

uint32_t be32(const unsigned char* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

void put_be32(std::string& o, uint32_t v) {
  o.push_back((char)(v >> 24));
  o.push_back((char)(v >> 16));
  o.push_back((char)(v >> 8));
  o.push_back((char)v);
}

void put_chunk(std::string& o, const char* type, const std::string& data) {
  put_be32(o, (uint32_t)data.size());
  std::string td(type, 4);
  td += data;
  o += td;
  put_be32(o, (uint32_t)crc32(0L, (const Bytef*)td.data(), (uInt)td.size()));
}

int paeth(int a, int b, int c) {
  const int p = a + b - c;
  const int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

}  // namespace
}  // namespace rmh

using namespace rmh;

extern "C" {

const char* rmh_last_error(void) { return g_err.c_str(); }

#ifndef RMH_SOURCE_SHA
#define RMH_SOURCE_SHA "unknown"  // _build.py passes the sha256 of the host sources
#endif
const char* rmh_version(void) { return "burn_raymarching_amd host 0.1.0 src " RMH_SOURCE_SHA; }

void rmh_free(void* p) { std::free(p); }

int rmh_png_read(const char* path, int32_t* width, int32_t* height, uint8_t** rgb) {
  if (!path || !width || !height || !rgb) return fail(RMH_ERR_INVALID_ARG, "NULL argument");
  std::string f;
  if (!read_file(path, f)) return fail(RMH_ERR_IO, "cannot read %s", path);
  static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) return fail(RMH_ERR_FORMAT, "%s: not a PNG", path);
  const unsigned char* b = (const unsigned char*)f.data();
  size_t pos = 8;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::string idat;
  std::vector<unsigned char> plte;
  bool end = false;
  while (!end && pos + 12 <= f.size()) {
    const uint32_t len = be32(b + pos);
    if (pos + 12 + (size_t)len > f.size()) return fail(RMH_ERR_FORMAT, "%s: truncated chunk", path);
    const std::string type(f.data() + pos + 4, 4);
    const unsigned char* d = b + pos + 8;
    const uint32_t crc = be32(d + len);
    if ((uint32_t)crc32(0L, b + pos + 4, len + 4) != crc) return fail(RMH_ERR_FORMAT, "%s: bad CRC in %s", path,
                                                                       type.c_str());
    if (type == "IHDR") {
      if (len != 13) return fail(RMH_ERR_FORMAT, "%s: bad IHDR", path);
      w = be32(d);
      h = be32(d + 4);
      depth = d[8];
      ctype = d[9];
      interlace = d[12];
    } else if (type == "PLTE") {
      plte.assign(d, d + len);
    } else if (type == "IDAT") {
      idat.append((const char*)d, len);
    } else if (type == "IEND") {
      end = true;
    }
    pos += 12 + (size_t)len;
  }
  if (w == 0 || h == 0 || w > (1u << 15) || h > (1u << 15)) return fail(RMH_ERR_FORMAT, "%s: bad size", path);
  if (depth != 8) return fail(RMH_ERR_FORMAT, "%s: only 8-bit PNGs are supported (depth %d)", path, depth);
  if (interlace != 0) return fail(RMH_ERR_FORMAT, "%s: interlaced PNGs are not supported", path);
  int ch;
  switch (ctype) {
    case 0: ch = 1; break;
    case 2: ch = 3; break;
    case 3: ch = 1; break;
    case 4: ch = 2; break;
    case 6: ch = 4; break;
    default: return fail(RMH_ERR_FORMAT, "%s: colour type %d", path, ctype);
  }
  if (ctype == 3 && plte.size() < 3) return fail(RMH_ERR_FORMAT, "%s: palette image without PLTE", path);
  const size_t stride = (size_t)w * ch;
  std::vector<unsigned char> raw((stride + 1) * h);
  uLongf rawlen = (uLongf)raw.size();
  if (uncompress(raw.data(), &rawlen, (const Bytef*)idat.data(), (uLong)idat.size()) != Z_OK ||
      rawlen != raw.size())
    return fail(RMH_ERR_FORMAT, "%s: bad image data", path);
  std::vector<unsigned char> px(stride * h);
  for (uint32_t y = 0; y < h; ++y) {
    const unsigned char* src = raw.data() + y * (stride + 1);
    unsigned char* row = px.data() + y * stride;
    const unsigned char* up = y ? row - stride : nullptr;
    const int filter = src[0];
    ++src;
    for (size_t x = 0; x < stride; ++x) {
      const int a = x >= (size_t)ch ? row[x - ch] : 0;
      const int u = up ? up[x] : 0;
      const int c = (up && x >= (size_t)ch) ? up[x - ch] : 0;
      int v = src[x];
      switch (filter) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += u; break;
        case 3: v += (a + u) >> 1; break;
        case 4: v += paeth(a, u, c); break;
        default: return fail(RMH_ERR_FORMAT, "%s: bad filter %d", path, filter);
      }
      row[x] = (unsigned char)v;
    }
  }
  uint8_t* o = (uint8_t*)std::malloc((size_t)w * h * 3);
  if (!o) return fail(RMH_ERR_IO, "out of host memory");
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    const unsigned char* s = px.data() + i * ch;
    switch (ctype) {
      case 0:
      case 4: o[3 * i] = o[3 * i + 1] = o[3 * i + 2] = s[0]; break;
      case 2:
      case 6: o[3 * i] = s[0]; o[3 * i + 1] = s[1]; o[3 * i + 2] = s[2]; break;
      case 3: {
        const size_t k = 3 * (size_t)s[0];
        if (k + 2 >= plte.size()) {
          std::free(o);
          return fail(RMH_ERR_FORMAT, "%s: palette index out of range", path);
        }
        o[3 * i] = plte[k];
        o[3 * i + 1] = plte[k + 1];
        o[3 * i + 2] = plte[k + 2];
        break;
      }
    }
  }
  *width = (int32_t)w;
  *height = (int32_t)h;
  *rgb = o;
  return RMH_OK;
}

int rmh_png_write(const char* path, const uint8_t* rgb, int32_t width, int32_t height) {
  if (!path || !rgb || width < 1 || height < 1) return fail(RMH_ERR_INVALID_ARG, "bad PNG write arguments");
  const size_t stride = (size_t)width * 3;
  std::string raw;
  raw.reserve((stride + 1) * height);
  for (int32_t y = 0; y < height; ++y) {
    raw.push_back('\0');  // filter: None
    raw.append((const char*)rgb + y * stride, stride);
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::string z(zlen, '\0');
  if (compress2((Bytef*)&z[0], &zlen, (const Bytef*)raw.data(), (uLong)raw.size(), 6) != Z_OK)
    return fail(RMH_ERR_IO, "zlib compression failed");
  z.resize(zlen);
  std::string o("\x89PNG\r\n\x1a\n", 8);
  std::string ihdr;
  put_be32(ihdr, (uint32_t)width);
  put_be32(ihdr, (uint32_t)height);
  ihdr += std::string("\x08\x02\x00\x00\x00", 5);  // 8-bit RGB, deflate, adaptive, no interlace
  put_chunk(o, "IHDR", ihdr);
  put_chunk(o, "IDAT", z);
  put_chunk(o, "IEND", std::string());
  if (!write_file(path, o)) return fail(RMH_ERR_IO, "cannot write %s", path);
  return RMH_OK;
}

void rmh_srgb8_to_linear(const uint8_t* in, int64_t n, float* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = std::pow((float)in[i] / 255.0f, 2.2f);
}

void rmh_linear_to_srgb8(const float* in, int64_t n, uint8_t* out) {
  const float g = 1.0f / 2.2f;
  for (int64_t i = 0; i < n; ++i) {
    float y = std::pow(in[i], g);
    y = std::isnan(y) ? 0.0f : std::fmin(std::fmax(y, 0.0f), 1.0f) * 255.0f;  // Rust `as u8` saturates
    out[i] = (uint8_t)y;
  }
}

int rmh_image_load(const char* path, int32_t* width, int32_t* height, float** linear_rgb) {
  if (!linear_rgb) return fail(RMH_ERR_INVALID_ARG, "NULL argument");
  uint8_t* px = nullptr;
  int rc = rmh_png_read(path, width, height, &px);
  if (rc) return rc;
  const int64_t n = (int64_t)*width * *height * 3;
  float* o = (float*)std::malloc((size_t)n * sizeof(float));
  if (!o) {
    std::free(px);
    return fail(RMH_ERR_IO, "out of host memory");
  }
  rmh_srgb8_to_linear(px, n, o);
  std::free(px);
  *linear_rgb = o;
  return RMH_OK;
}

int rmh_image_save(const char* path, const float* linear_rgb, int32_t width, int32_t height) {
  if (!linear_rgb || width < 1 || height < 1) return fail(RMH_ERR_INVALID_ARG, "bad image");
  std::vector<uint8_t> px((size_t)width * height * 3);
  rmh_linear_to_srgb8(linear_rgb, (int64_t)px.size(), px.data());
  return rmh_png_write(path, px.data(), width, height);
}

int rmh_cameras_load(const char* path, rmh_camera_entry** cams, int32_t* count) {
  if (!path || !cams || !count) return fail(RMH_ERR_INVALID_ARG, "NULL argument");
  std::string text, err;
  if (!read_file(path, text)) return fail(RMH_ERR_IO, "cannot read %s", path);
  Json j;
  if (!json_parse(text, j, err)) return fail(RMH_ERR_FORMAT, "%s: %s", path, err.c_str());
  if (j.kind != Json::Array) return fail(RMH_ERR_FORMAT, "%s: expected an array of cameras", path);
  std::vector<rmh_camera_entry> out(j.arr.size());
  for (size_t i = 0; i < j.arr.size(); ++i) {
    const Json& c = j.arr[i];
    const Json* file = c.get("file");
    const Json* fov = c.get("fov");
    std::vector<float> org, tgt;
    if (!file || file->kind != Json::String || !fov || fov->kind != Json::Number || !num_array(c.get("origin"), org) ||
        !num_array(c.get("target"), tgt) || org.size() != 3 || tgt.size() != 3)
      return fail(RMH_ERR_FORMAT, "%s: camera %zu lacks file/origin[3]/target[3]/fov", path, i);
    if (file->str.size() >= RMH_PATH_MAX) return fail(RMH_ERR_FORMAT, "%s: file name too long", path);
    std::memset(&out[i], 0, sizeof out[i]);
    std::memcpy(out[i].file, file->str.c_str(), file->str.size() + 1);
    for (int k = 0; k < 3; ++k) {
      out[i].origin[k] = org[k];
      out[i].target[k] = tgt[k];
    }
    out[i].fov = (float)fov->num;
  }
  rmh_camera_entry* o = (rmh_camera_entry*)std::malloc(std::max<size_t>(1, out.size()) * sizeof(rmh_camera_entry));
  if (!o) return fail(RMH_ERR_IO, "out of host memory");
  if (!out.empty()) std::memcpy(o, out.data(), out.size() * sizeof(rmh_camera_entry));
  *cams = o;
  *count = (int32_t)out.size();
  return RMH_OK;
}

int rmh_cameras_save(const char* path, const rmh_camera_entry* cams, int32_t count) {
  if (!path || (count > 0 && !cams) || count < 0) return fail(RMH_ERR_INVALID_ARG, "bad arguments");
  auto vec3 = [](const float* v) {
    return "[\n      " + fmt_f32(v[0]) + ",\n      " + fmt_f32(v[1]) + ",\n      " + fmt_f32(v[2]) + "\n    ]";
  };
  std::string o = count ? "[" : "[]";
  for (int32_t i = 0; i < count; ++i) {
    o += i ? ",\n  {\n" : "\n  {\n";
    o += "    \"file\": \"" + json_escape(cams[i].file) + "\",\n";
    o += "    \"origin\": " + vec3(cams[i].origin) + ",\n";
    o += "    \"target\": " + vec3(cams[i].target) + ",\n";
    o += "    \"fov\": " + fmt_f32(cams[i].fov) + "\n  }";
  }
  if (count) o += "\n]";
  if (!write_file(path, o)) return fail(RMH_ERR_IO, "cannot write %s", path);
  return RMH_OK;
}

int rmh_scene_save(const char* path, int32_t M, const float* centers, const float* colors, const float* radii,
                   const float* light_dir, const float* ambient) {
  if (!path || M < 0 || (M > 0 && (!centers || !colors || !radii)) || !light_dir || !ambient)
    return fail(RMH_ERR_INVALID_ARG, "bad scene arguments");
  std::string o = "{\n  \"num_spheres\": " + std::to_string(M) + ",\n";
  put_f32_array(o, "centers", centers, 3 * (size_t)M, false);
  put_f32_array(o, "colors", colors, 3 * (size_t)M, false);
  put_f32_array(o, "radii", radii, (size_t)M, false);
  put_f32_array(o, "light_dir", light_dir, 3, false);
  put_f32_array(o, "ambient_intensity", ambient, 1, true);
  o += "}";
  if (!write_file(path, o)) return fail(RMH_ERR_IO, "cannot write %s", path);
  return RMH_OK;
}

int rmh_scene_load(const char* path, int32_t* num_spheres, float** centers, float** colors, float** radii,
                   float light_dir[3], float* ambient) {
  if (!path || !num_spheres || !centers || !colors || !radii || !light_dir || !ambient)
    return fail(RMH_ERR_INVALID_ARG, "NULL argument");
  std::string text, err;
  if (!read_file(path, text)) return fail(RMH_ERR_IO, "cannot read %s", path);
  Json j;
  if (!json_parse(text, j, err)) return fail(RMH_ERR_FORMAT, "%s: %s", path, err.c_str());
  const Json* n = j.get("num_spheres");
  std::vector<float> c, col, r, ld, amb;
  if (!n || n->kind != Json::Number || !num_array(j.get("centers"), c) || !num_array(j.get("colors"), col) ||
      !num_array(j.get("radii"), r) || !num_array(j.get("light_dir"), ld) ||
      !num_array(j.get("ambient_intensity"), amb))
    return fail(RMH_ERR_FORMAT, "%s: missing scene fields", path);
  const size_t M = (size_t)n->num;
  if (c.size() != 3 * M || col.size() != 3 * M || r.size() != M || ld.size() != 3 || amb.size() != 1)
    return fail(RMH_ERR_FORMAT, "%s: inconsistent array sizes for num_spheres=%zu", path, M);
  auto dup = [](const std::vector<float>& v) {
    float* p = (float*)std::malloc(std::max<size_t>(1, v.size()) * sizeof(float));
    if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(float));
    return p;
  };
  *centers = dup(c);
  *colors = dup(col);
  *radii = dup(r);
  for (int k = 0; k < 3; ++k) light_dir[k] = ld[k];
  *ambient = amb[0];
  *num_spheres = (int32_t)M;
  return RMH_OK;
}

}  // extern "C"
