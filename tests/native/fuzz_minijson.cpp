// Random-input loop for native/include/minijson.h under AddressSanitizer + UBSan (tests/test_native_sanitizers.py).
// minijson parses what the OCI runtime shim and node_validate read from outside: bundle config.json,
// CDI specs, API-server responses and watch events.
//   fuzz_minijson [iterations] [seed]
// Properties: parse never crashes or leaks on any byte string; whatever it accepts dumps to text that
// parses again to the same dump (so a rewritten config.json is valid JSON); generated documents round
// trip exactly.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "minijson.h"

using minijson::Value;

static uint64_t g_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
  uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static int rn(int n) { return (int)(rnd() % (uint64_t)n); }

static std::string rand_string() {
  static const char* pieces[] = {"a", "Z", "0", " ", "\"", "\\", "/", "\n", "\t", "\x01", "\x7f", "\xc3\xa9",
                                 "\xf0\x9f\x98\x80", "\xff", "{", "}", "[", "]", ":", ","};
  std::string s;
  for (int i = rn(12); i > 0; --i) s += pieces[rn(sizeof pieces / sizeof *pieces)];
  return s;
}

static Value gen(int depth) {
  switch (depth > 6 ? rn(4) : rn(6)) {
    case 0: return Value::null();
    case 1: return Value::boolean(rn(2));
    case 2: {
      static const char* nums[] = {"0", "-0", "1", "-12", "3.25", "1e10", "-2.5E-3", "123456789012345678901234567890",
                                   "0.000001", "1E+2"};
      return Value::number_text(nums[rn(10)]);
    }
    case 3: return Value::string(rand_string());
    case 4: {
      Value a = Value::array();
      for (int i = rn(5); i > 0; --i) a.push(gen(depth + 1));
      return a;
    }
    default: {
      Value o = Value::object();
      for (int i = rn(5); i > 0; --i) o.o.emplace_back(rand_string(), gen(depth + 1));
      return o;
    }
  }
}

static std::string mutate(std::string s) {
  static const char alphabet[] = "{}[]\",:\\u0123456789abcdefABCDEF.eE+- \n\ttrufalsn\x00\xff";
  for (int m = 1 + rn(4); m > 0; --m) {
    const size_t at = s.empty() ? 0 : (size_t)rn((int)s.size() + 1);
    switch (rn(5)) {
      case 0:
        if (!s.empty() && at < s.size()) s[at] = alphabet[rn(sizeof alphabet - 1)];
        break;
      case 1: s.insert(at, 1, alphabet[rn(sizeof alphabet - 1)]); break;
      case 2:
        if (!s.empty() && at < s.size()) s.erase(at, 1 + rn(8));
        break;
      case 3: s = s.substr(0, at); break;
      default:
        if (!s.empty()) s.insert(at, s.substr((size_t)rn((int)s.size()), 1 + rn(16)));
    }
  }
  return s;
}

static int g_fail = 0;
static void expect(bool ok, const char* what, const std::string& in) {
  if (ok) return;
  std::fprintf(stderr, "FAIL %s on input of %zu bytes: %.200s\n", what, in.size(), in.c_str());
  ++g_fail;
}

// Accepted text must dump to a fixpoint that parses again.
static void check_accepted(const std::string& in) {
  Value v;
  try {
    v = minijson::parse(in);
  } catch (const std::exception&) {
    return;
  }
  const std::string d1 = minijson::dump(v), d2 = minijson::dump(v, 2);
  try {
    expect(minijson::dump(minijson::parse(d1)) == d1, "dump fixpoint", in);
    expect(minijson::dump(minijson::parse(d2)) == d1, "indented dump fixpoint", in);
  } catch (const std::exception& e) {
    expect(false, e.what(), in);
  }
}

int main(int argc, char** argv) {
  const long iters = argc > 1 ? std::atol(argv[1]) : 20000;
  if (argc > 2) g_state ^= std::strtoull(argv[2], nullptr, 10);
  const std::vector<std::string> corpus = {
      "{\"ociVersion\":\"1.0.2\",\"process\":{\"env\":[\"PATH=/bin\",\"AMD_VISIBLE_DEVICES=all\"],\"user\":{\"uid\":0}},"
      "\"linux\":{\"devices\":[{\"path\":\"/dev/kfd\",\"type\":\"c\",\"major\":236,\"minor\":0}]}}",
      "{\"type\":\"MODIFIED\",\"object\":{\"kind\":\"Node\",\"metadata\":{\"name\":\"n1\",\"resourceVersion\":\"42\"},"
      "\"status\":{\"capacity\":{\"amd.com/gpu\":\"8\",\"cpu\":\"96\"}}}}",
      "{\"type\":\"ERROR\",\"object\":{\"kind\":\"Status\",\"code\":410,\"reason\":\"Expired\"}}",
      "[1,-0.5e-3,true,false,null,\"\\u00e9\\ud83d\\ude00\\n\",{},[]]",
      "\"\\ud800\"", "\"\\udc00\"", "\"\\ud800\\u0041\"", "[1.]", "[.5]", "[--1]", "[1e]", "[01]", "[-]", "[.]",
  };
  for (const auto& c : corpus) check_accepted(c);
  // the strict number grammar: these are not JSON and must be refused
  for (const char* bad : {"[1.]", "[.5]", "[--1]", "[1e]", "[-]", "[.]", "[1e+]", "[+1]", "\"\\ud800\"",
                          "\"\\udc00\"", "\"\\ud800\\u0041\""}) {
    bool refused = false;
    try {
      minijson::parse(bad);
    } catch (const std::exception&) {
      refused = true;
    }
    expect(refused, "invalid JSON accepted", bad);
  }
  // nesting: a bounded depth, never a stack overflow
  for (int depth : {100, 256, 257, 5000, 100000}) {
    const std::string deep = std::string(depth, '[') + std::string(depth, ']');
    check_accepted(deep);
    const std::string deepo = [&] {
      std::string s;
      for (int i = 0; i < depth; ++i) s += "{\"a\":";
      s += "1";
      s += std::string(depth, '}');
      return s;
    }();
    check_accepted(deepo);
  }
  for (long i = 0; i < iters; ++i) {
    const Value v = gen(0);
    const std::string d = minijson::dump(v);
    try {
      expect(minijson::dump(minijson::parse(d)) == d, "generated round trip", d);
    } catch (const std::exception& e) {
      expect(false, e.what(), d);
    }
    check_accepted(mutate(rn(3) ? d : corpus[rn((int)corpus.size())]));
    std::string junk;
    for (int n = rn(64); n > 0; --n) junk += (char)rn(256);
    check_accepted(junk);
    if (g_fail > 20) break;
  }
  std::printf("{\"fuzz\":\"minijson\",\"iterations\":%ld,\"failures\":%d}\n", iters, g_fail);
  return g_fail ? 1 : 0;
}
