// json.h - minimal JSON DOM + parser for contents.json (the reference uses
// rapidjson: libVeles/src/main_file_loader.cc:42-180).
#pragma once
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace veles_rt {

struct Json {
  enum Type { Null, Bool, Number, String, Array, Object } type = Null;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<Json> arr;
  std::map<std::string, Json> obj;

  bool has(const std::string& k) const { return type == Object && obj.count(k); }
  const Json& operator[](const std::string& k) const {
    auto it = obj.find(k);
    if (it == obj.end()) throw std::runtime_error("json: missing key " + k);
    return it->second;
  }
  const Json& operator[](size_t i) const { return arr.at(i); }
  size_t size() const { return type == Array ? arr.size() : obj.size(); }

  static Json parse(const std::string& text) {
    size_t p = 0;
    Json j = parse_value(text, p);
    skip(text, p);
    if (p != text.size()) throw std::runtime_error("json: trailing data");
    return j;
  }

 private:
  static void skip(const std::string& s, size_t& p) {
    while (p < s.size() && (s[p] == ' ' || s[p] == '\n' || s[p] == '\t' ||
                            s[p] == '\r'))
      ++p;
  }
  static Json parse_value(const std::string& s, size_t& p) {
    skip(s, p);
    if (p >= s.size()) throw std::runtime_error("json: unexpected end");
    Json j;
    char c = s[p];
    if (c == '{') {
      j.type = Object;
      ++p;
      skip(s, p);
      if (s[p] == '}') { ++p; return j; }
      while (true) {
        skip(s, p);
        Json key = parse_value(s, p);
        skip(s, p);
        if (s[p] != ':') throw std::runtime_error("json: expected ':'");
        ++p;
        j.obj[key.str] = parse_value(s, p);
        skip(s, p);
        if (s[p] == ',') { ++p; continue; }
        if (s[p] == '}') { ++p; break; }
        throw std::runtime_error("json: expected ',' or '}'");
      }
    } else if (c == '[') {
      j.type = Array;
      ++p;
      skip(s, p);
      if (s[p] == ']') { ++p; return j; }
      while (true) {
        j.arr.push_back(parse_value(s, p));
        skip(s, p);
        if (s[p] == ',') { ++p; continue; }
        if (s[p] == ']') { ++p; break; }
        throw std::runtime_error("json: expected ',' or ']'");
      }
    } else if (c == '"') {
      j.type = String;
      ++p;
      while (p < s.size() && s[p] != '"') {
        if (s[p] == '\\') {
          ++p;
          char e = s[p];
          if (e == 'n') j.str += '\n';
          else if (e == 't') j.str += '\t';
          else if (e == 'u') { j.str += '?'; p += 4; }
          else j.str += e;
          ++p;
        } else {
          j.str += s[p++];
        }
      }
      ++p;
    } else if (s.compare(p, 4, "true") == 0) {
      j.type = Bool; j.b = true; p += 4;
    } else if (s.compare(p, 5, "false") == 0) {
      j.type = Bool; j.b = false; p += 5;
    } else if (s.compare(p, 4, "null") == 0) {
      j.type = Null; p += 4;
    } else {
      j.type = Number;
      char* end = nullptr;
      j.num = std::strtod(s.c_str() + p, &end);
      if (end == s.c_str() + p) throw std::runtime_error("json: bad token");
      p = end - s.c_str();
    }
    return j;
  }
};

}  // namespace veles_rt
