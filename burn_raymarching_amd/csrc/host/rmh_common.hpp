// Internal helpers shared by the librm_host.so sources (include/rm_host.h is the API).
#pragma once

#include <cstdarg>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "rm_host.h"

namespace rmh {

// Records the error text for rmh_last_error() and returns `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

bool read_file(const std::string& path, std::string& out);
bool write_file(const std::string& path, const std::string& data);
bool make_parent_dirs(const std::string& path);
bool make_dirs(const std::string& dir);
std::string dirname_of(const std::string& path);
std::string join_path(const std::string& dir, const std::string& name);

// ---- minimal JSON (RFC 8259 subset: no \u surrogate pairs beyond the BMP) ----------------
struct Json {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  double num = 0.0;
  std::string str;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;  // insertion order kept

  const Json* get(const std::string& key) const;
};
// Parses `text`; on error returns false and sets `err`.
bool json_parse(const std::string& text, Json& out, std::string& err);

// serde_json / ryu formatting of an f32 (shortest round trip, "1.0" for integral values).
std::string fmt_f32(float x);

// sigmoid / softplus(beta = 1) in f32, scene.rs:41-45 (softplus without the +0.01).
float sigmoid_f32(float x);
float softplus_f32(float x);

}  // namespace rmh
