// jubaconv: offline converter debugger, native (reference C34,
// jubatus/server/cmd/jubaconv.cpp:47-198).
//
// stdin JSON -> datum -> feature vector. -i json|datum, -o json|datum|fv,
// -c server_config.json (its "converter" section). JSON -> datum flattening
// (the core json_converter, EXTERNAL; parity unpinned, same rules as the
// Python twin jubatus_amd/cmd/jubaconv.py): object keys join as "/a/b", array
// elements as "/a[0]", strings go to string_values, numbers to num_values,
// booleans to num_values as 1 / 0, nulls are skipped. fv lines are
// "<feature>: <value>" (%g) from the native wide converter
// (csrc/native/jb_hostfv_wide.hpp: the feature names and values of the Python
// converter; values print as the float32 the models store). JSON output is
// Python's json.dumps(indent=2) byte for byte.
// A converter outside the wide rule set (filters, binary rules, plug-ins,
// regexp matchers) runs the Python twin instead: decided from -c before
// stdin is read, so the input goes to it untouched.
#include <stdio.h>
#include <unistd.h>

#include <charconv>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "jb_cmd.hpp"
#include "jb_server_common.hpp"
#include "jb_wide_rules.hpp"

namespace {

using jb::val::Value;

// ------------------------------------------------ Python json.dumps(indent=2)
// repr(float): shortest round-trip digits, fixed notation for decimal
// exponents in [-4, 16), scientific otherwise (exponent with sign and at
// least two digits), ".0" on integral fixed values
std::string py_float(double x) {
  if (x != x) return "NaN";
  if (x == INFINITY) return "Infinity";
  if (x == -INFINITY) return "-Infinity";
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
  std::string s(buf, r.ptr);
  const size_t e = s.find('e');
  std::string mant = s.substr(0, e);
  const int exp = atoi(s.c_str() + e + 1);
  std::string sign;
  if (mant[0] == '-') { sign = "-"; mant = mant.substr(1); }
  std::string digits;
  for (char c : mant)
    if (c != '.') digits += c;
  if (exp < -4 || exp >= 16) {
    std::string o = sign + digits.substr(0, 1);
    if (digits.size() > 1) o += "." + digits.substr(1);
    char eb[16];
    snprintf(eb, sizeof eb, "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
    return o + eb;
  }
  std::string o;
  if (exp < 0) {
    o = "0." + std::string((size_t)(-exp - 1), '0') + digits;
  } else if ((size_t)exp + 1 >= digits.size()) {
    o = digits + std::string((size_t)exp + 1 - digits.size(), '0') + ".0";
  } else {
    o = digits.substr(0, (size_t)exp + 1) + "." + digits.substr((size_t)exp + 1);
  }
  return sign + o;
}

// ensure_ascii string: \uXXXX for non-ASCII (surrogate pairs past the BMP)
std::string py_str(const std::string& s) {
  std::string o = "\"";
  char u[16];
  for (size_t i = 0; i < s.size();) {
    const uint8_t c = (uint8_t)s[i];
    uint32_t cp = c;
    size_t n = 1;
    if (c >= 0x80) {
      n = c >= 0xf0 ? 4 : c >= 0xe0 ? 3 : c >= 0xc0 ? 2 : 1;
      cp = n == 4 ? c & 7 : n == 3 ? c & 15 : n == 2 ? c & 31 : 0xfffd;
      for (size_t k = 1; k < n && i + k < s.size(); ++k) cp = (cp << 6) | ((uint8_t)s[i + k] & 63);
    }
    i += n;
    switch (cp) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '\b': o += "\\b"; continue;
      case '\f': o += "\\f"; continue;
      default: break;
    }
    if (cp >= 0x20 && cp < 0x7f) {
      o += (char)cp;
    } else if (cp < 0x10000) {
      snprintf(u, sizeof u, "\\u%04x", cp);
      o += u;
    } else {
      cp -= 0x10000;
      snprintf(u, sizeof u, "\\u%04x\\u%04x", 0xd800 + (cp >> 10), 0xdc00 + (cp & 0x3ff));
      o += u;
    }
  }
  return o + "\"";
}

void dump(const Value& v, int ind, std::string* o) {
  const std::string pad((size_t)(ind + 2), ' '), end((size_t)ind, ' ');
  switch (v.kind) {
    case Value::NIL: *o += "null"; break;
    case Value::BOOL: *o += v.b ? "true" : "false"; break;
    case Value::INT: *o += std::to_string(v.i); break;
    case Value::UINT: *o += std::to_string(v.u); break;
    case Value::DBL: *o += py_float(v.d); break;
    case Value::STR: case Value::BIN: *o += py_str(v.s); break;
    case Value::ARR:
      if (v.a.empty()) { *o += "[]"; break; }
      *o += "[\n";
      for (size_t i = 0; i < v.a.size(); ++i) {
        *o += pad;
        dump(v.a[i], ind + 2, o);
        *o += i + 1 < v.a.size() ? ",\n" : "\n";
      }
      *o += end + "]";
      break;
    case Value::MAP:
      if (v.o.empty()) { *o += "{}"; break; }
      *o += "{\n";
      for (size_t i = 0; i < v.o.size(); ++i) {
        *o += pad + py_str(v.o[i].first) + ": ";
        dump(v.o[i].second, ind + 2, o);
        *o += i + 1 < v.o.size() ? ",\n" : "\n";
      }
      *o += end + "}";
      break;
  }
}

// ------------------------------------------------------------------- datum
struct Datum {
  std::vector<std::pair<std::string, std::string>> str;
  std::vector<std::pair<std::string, double>> num;
  std::vector<std::pair<std::string, std::string>> bin;
};

void json_to_datum(const Value& v, const std::string& prefix, Datum* d) {
  switch (v.kind) {
    case Value::MAP:
      for (const auto& kv : v.o) json_to_datum(kv.second, prefix + "/" + kv.first, d);
      break;
    case Value::ARR:
      for (size_t i = 0; i < v.a.size(); ++i) json_to_datum(v.a[i], prefix + "[" + std::to_string(i) + "]", d);
      break;
    case Value::BOOL: d->num.emplace_back(prefix, v.b ? 1.0 : 0.0); break;
    case Value::INT: case Value::UINT: case Value::DBL: d->num.emplace_back(prefix, v.num()); break;
    case Value::STR: case Value::BIN: d->str.emplace_back(prefix, v.s); break;
    case Value::NIL: break;
  }
}

// {"string_values": [[k, v]...], "num_values": [[k, x]...], "binary_values": [[k, b]...]}
Datum datum_from_json(const Value& v) {
  Datum d;
  auto pairs = [&](const char* key, auto fn) {
    const Value* l = v.get(key);
    if (!l || l->kind != Value::ARR) return;
    for (const Value& p : l->a) {
      if (p.kind != Value::ARR || p.a.size() != 2) throw std::runtime_error(std::string("bad ") + key);
      fn(p.a[0], p.a[1]);
    }
  };
  auto text = [](const Value& x) {
    if (x.is_str()) return x.s;
    std::string o;
    dump(x, 0, &o);
    return o;
  };
  pairs("string_values", [&](const Value& k, const Value& x) { d.str.emplace_back(text(k), text(x)); });
  pairs("num_values", [&](const Value& k, const Value& x) {
    if (!x.is_num()) throw std::runtime_error("bad num_values");
    d.num.emplace_back(text(k), x.num());
  });
  pairs("binary_values", [&](const Value& k, const Value& x) { d.bin.emplace_back(text(k), text(x)); });
  return d;
}

Value datum_to_json(const Datum& d) {
  auto S = [](const std::string& s) { Value v; v.kind = Value::STR; v.s = s; return v; };
  auto pair = [](Value a, Value b) { Value v; v.kind = Value::ARR; v.a = {std::move(a), std::move(b)}; return v; };
  Value out, sv, nv, bv;
  out.kind = Value::MAP;
  sv.kind = nv.kind = bv.kind = Value::ARR;
  for (const auto& p : d.str) sv.a.push_back(pair(S(p.first), S(p.second)));
  for (const auto& p : d.num) {
    Value x;
    x.kind = Value::DBL;
    x.d = p.second;
    nv.a.push_back(pair(S(p.first), x));
  }
  for (const auto& p : d.bin) bv.a.push_back(pair(S(p.first), S(p.second)));
  out.o = {{"string_values", sv}, {"num_values", nv}, {"binary_values", bv}};
  return out;
}

// the datum as a one-element msgpack list<datum> body
std::string datum_body(const Datum& d) {
  jb::val::MsgpackWriter w;
  w.arr(1);
  w.arr(3);
  w.arr(d.str.size());
  for (const auto& p : d.str) { w.arr(2); w.raw(p.first); w.raw(p.second); }
  w.arr(d.num.size());
  for (const auto& p : d.num) { w.arr(2); w.raw(p.first); w.dbl(p.second); }
  w.arr(d.bin.size());
  for (const auto& p : d.bin) { w.arr(2); w.raw(p.first); w.bin(p.second.data(), p.second.size()); }
  return w.out;
}

struct Wide {
  std::vector<jb::HostRule> s, n, c;
  std::string blob;
  uint64_t H = 1ull << 20;
  bool global = false;
};
std::shared_ptr<jb::WideExt> ext;   // plug-ins, filters, binary rules of the converter

[[noreturn]] void run_python(char** argv) {
  std::string here(256, '\0');
  ssize_t k = readlink("/proc/self/exe", &here[0], here.size() - 1);
  here.resize(k > 0 ? (size_t)k : 0);
  // <root>/jubatus_amd/native_bin/jubaconv -> <root>
  for (int i = 0; i < 3 && !here.empty(); ++i) here = here.substr(0, here.rfind('/'));
  const char* pp = getenv("PYTHONPATH");
  const std::string path = here + (pp && *pp ? std::string(":") + pp : std::string());
  setenv("PYTHONPATH", path.c_str(), 1);
  std::vector<char*> args{(char*)"python3", (char*)"-m", (char*)"jubatus_amd.cmd.jubaconv"};
  for (char** a = argv + 1; *a; ++a) args.push_back(*a);
  args.push_back(nullptr);
  execvp("python3", args.data());
  perror("jubaconv: python3");
  _exit(127);
}

}  // namespace

int main(int argc, char** argv) {
  jb::cmd::Flags f("jubaconv");
  f.add('i', "input-format", "json", "input format: json|datum");
  f.add('o', "output-format", "fv", "output format: json|datum|fv");
  f.add('c', "conf", "", "server config file (its converter section)");
  int code = 0;
  if (!f.parse(argc, argv, &code)) return code;
  const std::string in = f.get("input-format"), out = f.get("output-format");
  if ((in != "json" && in != "datum") || (out != "json" && out != "datum" && out != "fv")) {
    f.usage(stderr);
    return 1;
  }
  // the converter first (before stdin): one the wide set does not take goes to Python
  std::unique_ptr<jb::HostFvWide> hw;
  Wide w;
  if (out == "fv" && !f.get("conf").empty()) {
    std::ifstream cf(f.get("conf"), std::ios::binary);
    if (!cf) {
      fprintf(stderr, "cannot open converter config file: %s\n", f.get("conf").c_str());
      return -1 & 0xff;
    }
    std::stringstream ss;
    ss << cf.rdbuf();
    Value conf;
    try {
      conf = jb::val::parse_json(ss.str());
    } catch (const std::exception&) {
      run_python(argv);      // the Python tool reports the config error its own way
    }
    const Value* conv = conf.get("converter");
    Value empty;
    empty.kind = Value::MAP;
    std::string why;
    if (!jb::row::build_wide_rules(conv && conv->kind == Value::MAP ? *conv : empty, &w.s, &w.n, &w.c, &w.blob,
                                   &w.H, &w.global, &why, &ext))
      run_python(argv);
    hw.reset(new jb::HostFvWide((const uint8_t*)w.s.data(), (int)w.s.size(), (const uint8_t*)w.n.data(),
                                (int)w.n.size(), (const uint8_t*)w.c.data(), (int)w.c.size() / 2,
                                (const uint8_t*)w.blob.data(), w.blob.size(), w.H));
    hw->set_ext(ext);
  }
  std::stringstream ss;
  ss << std::cin.rdbuf();
  Value data;
  try {
    data = jb::val::parse_json(ss.str());
  } catch (const std::exception&) {
    fprintf(stderr, "invalid %s format\n", in.c_str());
    return 255;
  }
  std::string o;
  if (out == "json") {
    if (in != "json") {
      fprintf(stderr, "invalid input-output type: %s -> json\n", in.c_str());
      return 255;
    }
    dump(data, 0, &o);
    printf("%s\n", o.c_str());
    return 0;
  }
  Datum d;
  try {
    if (in == "datum") d = datum_from_json(data);
    else json_to_datum(data, "", &d);
  } catch (const std::exception& e) {
    fprintf(stderr, "invalid datum: %s\n", e.what());
    return 255;
  }
  if (out == "datum") {
    dump(datum_to_json(d), 0, &o);
    printf("%s\n", o.c_str());
    return 0;
  }
  if (!hw) {
    fprintf(stderr, "specify converter config with -c flag\n");
    return 255;
  }
  // empty document statistics: a fresh converter's convert() (no update)
  std::vector<int64_t> df, diff;
  int64_t counts[4] = {0, 0, 0, 0};
  if (hw->needs_weights()) {
    df.assign(w.H, 0);
    diff.assign(w.H, 0);
  }
  hw->set_weights(df.empty() ? nullptr : df.data(), diff.empty() ? nullptr : diff.data(), counts);
  const std::string body = datum_body(d);
  std::vector<int32_t> idx(256);
  std::vector<float> val(idx.size());
  std::string names;
  std::vector<int64_t> name_end;
  int64_t rp[2] = {0, 0};
  int rc;
  for (;;) {
    int64_t n = 0, slots = 0;
    names.clear();
    name_end.clear();
    hw->set_sinks(&names, &name_end, nullptr);
    rc = hw->hash_body((const uint8_t*)body.data(), body.size(), idx.data(), val.data(), rp, 1,
                       (int64_t)idx.size(), &n, &slots, false);
    if (rc != 2) break;
    idx.resize(idx.size() * 4);
    val.resize(idx.size());
  }
  if (rc) {
    fprintf(stderr, "conversion failed\n");
    return 255;
  }
  int64_t st = 0;
  for (int64_t i = 0; i < rp[1]; ++i) {
    printf("%.*s: %g\n", (int)(name_end[(size_t)i] - st), names.data() + st, (double)val[(size_t)i]);
    st = name_end[(size_t)i];
  }
  return 0;
}
