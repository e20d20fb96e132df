// toml.cpp — a small TOML reader covering what the reference's scene files use
// (scene-definitions/*.toml, parsed there by the `toml` crate into the serde schema of
// src/configuration.rs): [dotted.tables], [[arrays.of.tables]], key = value with
// floats, integers, booleans, basic strings, arrays, inline tables, and comments.
#include <cctype>
#include <cstdlib>
#include <string>

#include "host_internal.h"

namespace grt_host {
namespace {

struct Parser {
  const std::string& s;
  size_t p = 0;
  int line = 1;
  std::string err;
  explicit Parser(const std::string& text) : s(text) {}

  bool fail(const std::string& m) {
    err = "line " + std::to_string(line) + ": " + m;
    return false;
  }
  void skip_ws() {
    while (p < s.size() && (s[p] == ' ' || s[p] == '\t')) ++p;
  }
  void skip_comment() {
    if (p < s.size() && s[p] == '#')
      while (p < s.size() && s[p] != '\n') ++p;
  }
  void skip_ws_nl() {  // inside arrays: whitespace, newlines, comments
    for (;;) {
      skip_ws();
      skip_comment();
      if (p < s.size() && (s[p] == '\n' || s[p] == '\r')) {
        if (s[p] == '\n') ++line;
        ++p;
        continue;
      }
      break;
    }
  }
  bool parse_key(std::string& k) {
    skip_ws();
    if (p < s.size() && (s[p] == '"' || s[p] == '\'')) {
      char q = s[p++];
      size_t st = p;
      while (p < s.size() && s[p] != q) ++p;
      if (p >= s.size()) return fail("unterminated quoted key");
      k = s.substr(st, p - st);
      ++p;
      return true;
    }
    size_t st = p;
    while (p < s.size() && (std::isalnum((unsigned char)s[p]) || s[p] == '_' || s[p] == '-')) ++p;
    if (p == st) return fail("expected a key");
    k = s.substr(st, p - st);
    return true;
  }
  bool parse_dotted(std::vector<std::string>& keys) {
    keys.clear();
    for (;;) {
      std::string k;
      if (!parse_key(k)) return false;
      keys.push_back(k);
      skip_ws();
      if (p < s.size() && s[p] == '.') {
        ++p;
        continue;
      }
      return true;
    }
  }
  bool parse_string(std::string& out) {
    char q = s[p++];
    out.clear();
    while (p < s.size() && s[p] != q) {
      if (q == '"' && s[p] == '\\' && p + 1 < s.size()) {
        char e = s[p + 1];
        out += (e == 'n') ? '\n' : (e == 't') ? '\t' : e;
        p += 2;
        continue;
      }
      if (s[p] == '\n') return fail("newline in string");
      out += s[p++];
    }
    if (p >= s.size()) return fail("unterminated string");
    ++p;
    return true;
  }
  bool parse_value(std::shared_ptr<TomlValue>& v) {
    skip_ws();
    if (p >= s.size()) return fail("expected a value");
    v = std::make_shared<TomlValue>();
    char c = s[p];
    if (c == '"' || c == '\'') {
      v->kind = TomlValue::String;
      return parse_string(v->s);
    }
    if (c == '[') {
      ++p;
      v->kind = TomlValue::Array;
      skip_ws_nl();
      if (p < s.size() && s[p] == ']') {
        ++p;
        return true;
      }
      for (;;) {
        std::shared_ptr<TomlValue> e;
        if (!parse_value(e)) return false;
        v->arr.push_back(e);
        skip_ws_nl();
        if (p < s.size() && s[p] == ',') {
          ++p;
          skip_ws_nl();
          if (p < s.size() && s[p] == ']') {
            ++p;
            return true;
          }
          continue;
        }
        if (p < s.size() && s[p] == ']') {
          ++p;
          return true;
        }
        return fail("expected ',' or ']' in array");
      }
    }
    if (c == '{') {
      ++p;
      v->kind = TomlValue::Table;
      skip_ws();
      if (p < s.size() && s[p] == '}') {
        ++p;
        return true;
      }
      for (;;) {
        std::vector<std::string> keys;
        if (!parse_dotted(keys)) return false;
        skip_ws();
        if (p >= s.size() || s[p] != '=') return fail("expected '=' in inline table");
        ++p;
        std::shared_ptr<TomlValue> e;
        if (!parse_value(e)) return false;
        TomlTable* t = &v->table;
        for (size_t i = 0; i + 1 < keys.size(); ++i) {
          auto& slot = (*t)[keys[i]];
          if (!slot) slot = std::make_shared<TomlValue>();
          t = &slot->table;
        }
        (*t)[keys.back()] = e;
        skip_ws();
        if (p < s.size() && s[p] == ',') {
          ++p;
          continue;
        }
        if (p < s.size() && s[p] == '}') {
          ++p;
          return true;
        }
        return fail("expected ',' or '}' in inline table");
      }
    }
    size_t st = p;
    while (p < s.size() && !std::isspace((unsigned char)s[p]) && s[p] != ',' && s[p] != ']' && s[p] != '}' &&
           s[p] != '#')
      ++p;
    std::string tok = s.substr(st, p - st);
    if (tok == "true" || tok == "false") {
      v->kind = TomlValue::Bool;
      v->b = tok == "true";
      return true;
    }
    std::string clean;
    for (char ch : tok)
      if (ch != '_') clean += ch;
    if (clean.empty()) return fail("empty value");
    bool is_float = clean.find_first_of(".eE") != std::string::npos || clean == "inf" || clean == "+inf" ||
                    clean == "-inf" || clean == "nan" || clean == "+nan" || clean == "-nan";
    char* end = nullptr;
    if (is_float) {
      v->kind = TomlValue::Float;
      v->f = std::strtod(clean.c_str(), &end);
    } else {
      v->kind = TomlValue::Int;
      v->i = std::strtoll(clean.c_str(), &end, 10);
      v->f = (double)v->i;
    }
    if (!end || *end) return fail("invalid value '" + tok + "'");
    return true;
  }
  TomlTable* descend(TomlTable& root, const std::vector<std::string>& keys, bool array_last) {
    TomlTable* t = &root;
    for (size_t i = 0; i < keys.size(); ++i) {
      bool last = i + 1 == keys.size();
      auto& slot = (*t)[keys[i]];
      if (last && array_last) {
        if (!slot) {
          slot = std::make_shared<TomlValue>();
          slot->kind = TomlValue::TableArray;
        }
        if (slot->kind != TomlValue::TableArray) {
          fail("'" + keys[i] + "' is not an array of tables");
          return nullptr;
        }
        auto e = std::make_shared<TomlValue>();
        e->kind = TomlValue::Table;
        slot->arr.push_back(e);
        return &e->table;
      }
      if (!slot) {
        slot = std::make_shared<TomlValue>();
        slot->kind = TomlValue::Table;
      }
      if (slot->kind == TomlValue::TableArray) {
        if (slot->arr.empty()) {
          fail("empty array of tables");
          return nullptr;
        }
        t = &slot->arr.back()->table;
      } else if (slot->kind == TomlValue::Table) {
        t = &slot->table;
      } else {
        fail("'" + keys[i] + "' is not a table");
        return nullptr;
      }
    }
    return t;
  }
  bool run(TomlTable& root) {
    TomlTable* cur = &root;
    while (p < s.size()) {
      skip_ws();
      skip_comment();
      if (p >= s.size()) break;
      if (s[p] == '\n' || s[p] == '\r') {
        if (s[p] == '\n') ++line;
        ++p;
        continue;
      }
      if (s[p] == '[') {
        bool arr = p + 1 < s.size() && s[p + 1] == '[';
        p += arr ? 2 : 1;
        std::vector<std::string> keys;
        if (!parse_dotted(keys)) return false;
        skip_ws();
        if (arr) {
          if (s.compare(p, 2, "]]") != 0) return fail("expected ']]'");
          p += 2;
        } else {
          if (p >= s.size() || s[p] != ']') return fail("expected ']'");
          ++p;
        }
        cur = descend(root, keys, arr);
        if (!cur) return false;
        continue;
      }
      std::vector<std::string> keys;
      if (!parse_dotted(keys)) return false;
      skip_ws();
      if (p >= s.size() || s[p] != '=') return fail("expected '='");
      ++p;
      std::shared_ptr<TomlValue> v;
      if (!parse_value(v)) return false;
      TomlTable* t = cur;
      for (size_t i = 0; i + 1 < keys.size(); ++i) {
        auto& slot = (*t)[keys[i]];
        if (!slot) {
          slot = std::make_shared<TomlValue>();
          slot->kind = TomlValue::Table;
        }
        t = &slot->table;
      }
      if (t->count(keys.back())) return fail("duplicate key '" + keys.back() + "'");
      (*t)[keys.back()] = v;
      skip_ws();
      skip_comment();
      if (p < s.size() && s[p] != '\n' && s[p] != '\r') return fail("trailing characters after value");
    }
    return true;
  }
};

}  // namespace

bool toml_parse(const std::string& text, TomlTable& root, std::string& err) {
  Parser ps(text);
  if (!ps.run(root)) {
    err = ps.err;
    return false;
  }
  return true;
}

}  // namespace grt_host
