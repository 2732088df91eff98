// The launcher <-> worker line protocol of amd-gemm-validate (native/hip/gemm_validate.cpp) and the
// option / shape lists it parses. Host-only C++ (no HIP types) so the sanitizer tier builds it
// without a GPU toolchain and fuzzes every parser here (tests/native/fuzz_protocol.cpp): the
// launcher reads these lines from child processes, the worker reads its plan from the launcher.
//
// Worker -> launcher (the worker's stdout):
//   S <hip device count> <bdf> <gcn arch> <cus> <lds per block>   after HIP init
//   H <0|1>                                                       hip-smoke result
//   W <set>                                                       at the set's rendezvous
//   R <set> <33 result fields> <bad-tile list> <error...>         the set's result (fmt_result_line)
// Launcher -> worker: "P <id>:<dtype>:<m>x<n>x<k>:<gpus>;..." once, then "g" per rendezvous.
//
// Every number is parsed with a range-checked conversion (strtoll / strtod on one whitespace-delimited
// token): a field out of range or a token that is not a number fails the line instead of being
// truncated or wrapped, so a corrupted pipe reads as a lost worker, never as a result.
#pragma once

#include <cerrno>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <climits>
#include <string>
#include <vector>

namespace vproto {

struct Shape {
  int m, n, k;
};

struct Options {
  int iters = 50, warmup = 5, check_rows = 32;
  int inject_tm = -1, inject_tn = -1;   // --inject-fault TM,TN[,DELTA]: perturb one element of that tile
  double inject_delta = 64.0;
  double stabilise_max_s = 6.0;
  double min_window_ms = 100.0;   // the timed loop covers at least this much GPU time
  double ramp_ms = 60.0;          // re-ramp after the rendezvous: at least this much GPU time (profiles/r5_ramp)
  double pre_idle_ms = 0.0;       // test hook: host idle after the rendezvous
  bool stabilise = true;
};

// The ABFT check of the checked dispatch (gemm_abft.hip): every output element covered, a failing
// tile named with the workgroup that computed it and, from that dispatch's placement record, the
// XCD and CU it ran on.
struct AbftOut {
  bool ran = false;
  int variant = -1, tile_m = 0, tile_n = 0, bad_tiles = 0;
  double worst_ratio = 0, checked_fraction = 0, check_ms = 0, abft_ms = 0;
  double dispatch_ms = 0, rows_ms = 0;   // the checked phase's other parts: poison + recorded dispatch, sampled rows
  // the first bad tile (row-major order): its workgroup (piece 0), round, XCD (-1: pieces of a split-K
  // tile ran on different XCDs, see `list`) and hardware id fields
  int tm = -1, tn = -1, wg = -1, round = -1, xcd = -1, se = -1, sh = -1, cu = -1;
  std::string list;   // up to 8 bad tiles "tm.tn.xcd" joined by ';' ("-": none)
};

struct Result {
  int device = 0;
  Shape s{};
  double tflops = 0, ms = 0, max_rel_err = 0, stab_spread = -1, stab_ms = 0, probe_ms = 0;
  int stab_dispatches = 0, iters = 0, ramp = 0;
  bool launched = false, ok = false, oom = false;
  size_t need_bytes = 0, free_bytes = 0;
  AbftOut abft;
  std::string error;
};

// --- tokens ----------------------------------------------------------------------------------
// The next whitespace-delimited token at or after `pos`; false at the end of the line.
inline bool next_token(const std::string& s, size_t& pos, std::string& tok) {
  while (pos < s.size() && (s[pos] == ' ' || s[pos] == '\t' || s[pos] == '\r' || s[pos] == '\n')) ++pos;
  if (pos >= s.size()) return false;
  const size_t b = pos;
  while (pos < s.size() && s[pos] != ' ' && s[pos] != '\t' && s[pos] != '\r' && s[pos] != '\n') ++pos;
  tok.assign(s, b, pos - b);
  return true;
}

inline bool to_ll(const std::string& t, long long lo, long long hi, long long& v) {
  if (t.empty()) return false;
  errno = 0;
  char* end = nullptr;
  const long long x = std::strtoll(t.c_str(), &end, 10);
  if (errno != 0 || end != t.c_str() + t.size() || x < lo || x > hi) return false;
  v = x;
  return true;
}

inline bool to_int(const std::string& t, int& v) {
  long long x = 0;
  if (!to_ll(t, INT_MIN, INT_MAX, x)) return false;
  v = (int)x;
  return true;
}

inline bool to_size(const std::string& t, size_t& v) {
  long long x = 0;
  if (!to_ll(t, 0, LLONG_MAX, x)) return false;
  v = (size_t)x;
  return true;
}

inline bool to_dbl(const std::string& t, double& v) {
  if (t.empty()) return false;
  char* end = nullptr;
  const double x = std::strtod(t.c_str(), &end);
  if (end != t.c_str() + t.size()) return false;
  v = x;
  return true;
}

// Reads the next token of `s` as the target's type. A small visitor over int / size_t / double / bool.
struct Reader {
  const std::string& s;
  size_t pos = 0;
  bool ok = true;
  std::string tok;
  bool take() { return ok && (ok = next_token(s, pos, tok)); }
  Reader& operator>>(int& v) {
    if (take()) ok = to_int(tok, v);
    return *this;
  }
  Reader& operator>>(size_t& v) {
    if (take()) ok = to_size(tok, v);
    return *this;
  }
  Reader& operator>>(double& v) {
    if (take()) ok = to_dbl(tok, v);
    return *this;
  }
  Reader& operator>>(bool& v) {
    int x = 0;
    if (take() && (ok = to_int(tok, x))) ok = (x == 0 || x == 1), v = x == 1;
    return *this;
  }
  Reader& operator>>(std::string& v) {
    if (take()) v = tok;
    return *this;
  }
};

// --- lists on the command line -----------------------------------------------------------------
// "8192,4096,16384x16384x1024": a square shape per bare number. A token that is neither is skipped.
inline std::vector<Shape> parse_shapes(const std::string& spec) {
  std::vector<Shape> out;
  size_t pos = 0;
  while (pos <= spec.size()) {
    const size_t c = spec.find(',', pos);
    const std::string t = spec.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
    if (!t.empty()) {
      std::vector<int> v;
      size_t q = 0;
      bool good = true;
      while (good && q <= t.size()) {
        const size_t x = t.find('x', q);
        int n = 0;
        good = to_int(t.substr(q, x == std::string::npos ? std::string::npos : x - q), n);
        if (good) v.push_back(n);
        if (x == std::string::npos) break;
        q = x + 1;
      }
      if (good && v.size() == 3) out.push_back({v[0], v[1], v[2]});
      else if (good && v.size() == 1) out.push_back({v[0], v[0], v[0]});
    }
    if (c == std::string::npos) break;
    pos = c + 1;
  }
  return out;
}

// parse_shapes, and whether every non-empty comma token of `spec` was a shape (a typo must not
// shrink the plan silently).
inline bool parse_shapes_strict(const std::string& spec, std::vector<Shape>& out) {
  out = parse_shapes(spec);
  size_t tokens = 0, pos = 0;
  while (pos <= spec.size()) {
    const size_t c = spec.find(',', pos);
    tokens += (c == std::string::npos ? spec.size() : c) > pos;
    if (c == std::string::npos) break;
    pos = c + 1;
  }
  return tokens == out.size() && !out.empty();
}

inline std::vector<int> parse_ints(const std::string& spec) {
  std::vector<int> out;
  for (const auto& s : parse_shapes(spec)) out.push_back(s.m);
  return out;
}

// A comma list of non-negative integers; false when any entry is not one (a UUID, say).
inline bool parse_index_list(const char* spec, std::vector<int>& out) {
  out.clear();
  const std::string s = spec ? spec : "";
  size_t pos = 0;
  while (pos <= s.size()) {
    const size_t c = s.find(',', pos);
    const std::string t = s.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
    if (!t.empty()) {
      long long v = 0;
      if (t[0] == '-' || t[0] == '+' || !to_ll(t, 0, INT_MAX, v)) return false;
      out.push_back((int)v);
    }
    if (c == std::string::npos) break;
    pos = c + 1;
  }
  return true;
}

// --- the worker's options (--worker-opts) ---------------------------------------------------------
inline std::string fmt_opts(const Options& o) {
  char buf[400];
  std::snprintf(buf, sizeof buf, "%d %d %d %.17g %.17g %.17g %.17g %d %d %d %.17g", o.iters, o.warmup, o.check_rows,
                o.stabilise_max_s, o.min_window_ms, o.ramp_ms, o.pre_idle_ms, o.stabilise ? 1 : 0, o.inject_tm,
                o.inject_tn, o.inject_delta);
  return buf;
}

inline bool parse_opts(const std::string& s, Options& o) {
  Options x;
  Reader r{s};
  r >> x.iters >> x.warmup >> x.check_rows >> x.stabilise_max_s >> x.min_window_ms >> x.ramp_ms >> x.pre_idle_ms >>
      x.stabilise >> x.inject_tm >> x.inject_tn >> x.inject_delta;
  std::string extra;
  if (!r.ok || next_token(s, r.pos, extra)) return false;
  o = x;
  return true;
}

// --- S: the worker's start line -----------------------------------------------------------------
struct StartLine {
  int ndev = 0;
  std::string bus, arch;
  int cus = 0;
  size_t lds = 0;
};

inline std::string fmt_start_line(const StartLine& l) {
  return "S " + std::to_string(l.ndev) + " " + (l.bus.empty() ? "-" : l.bus) + " " + (l.arch.empty() ? "-" : l.arch) +
         " " + std::to_string(l.cus) + " " + std::to_string(l.lds);
}

inline bool parse_start_line(const std::string& ln, StartLine& out) {
  StartLine l;
  Reader r{ln};
  std::string tag;
  r >> tag;
  if (!r.ok || tag != "S") return false;
  r >> l.ndev >> l.bus >> l.arch >> l.cus >> l.lds;
  if (!r.ok || l.bus.size() > 63 || l.arch.size() > 95) return false;
  out = l;
  return true;
}

// --- P: the worker's part of the plan ------------------------------------------------------------
struct PlanItem {
  int id = 0;
  std::string dtype;
  Shape s{};
  int set_size = 1;
};

inline std::string fmt_plan_item(const PlanItem& p) {
  return std::to_string(p.id) + ":" + p.dtype + ":" + std::to_string(p.s.m) + "x" + std::to_string(p.s.n) + "x" +
         std::to_string(p.s.k) + ":" + std::to_string(p.set_size);
}

inline bool parse_plan_item(const std::string& item, PlanItem& out) {
  // <id>:<dtype>:<m>x<n>x<k>:<gpus>
  std::vector<std::string> f;
  size_t pos = 0;
  while (pos <= item.size() && f.size() < 5) {
    const size_t c = item.find(':', pos);
    f.push_back(item.substr(pos, c == std::string::npos ? std::string::npos : c - pos));
    if (c == std::string::npos) break;
    pos = c + 1;
  }
  if (f.size() != 4 || f[1].empty() || f[1].size() > 31) return false;
  PlanItem p;
  p.dtype = f[1];
  const std::vector<Shape> sh = parse_shapes(f[2]);
  if (!to_int(f[0], p.id) || sh.size() != 1 || f[2].find('x') == std::string::npos || !to_int(f[3], p.set_size) ||
      p.set_size < 1)
    return false;
  p.s = sh[0];
  if (p.s.m <= 0 || p.s.n <= 0 || p.s.k <= 0) return false;
  out = p;
  return true;
}

// "P item;item;..." (the leading P optional); false if any item does not parse
inline bool parse_plan_line(const std::string& line, std::vector<PlanItem>& out) {
  std::string sets = line;
  if (!sets.empty() && sets[0] == 'P') sets.erase(0, 1);
  while (!sets.empty() && (sets.back() == '\n' || sets.back() == '\r' || sets.back() == ' ')) sets.pop_back();
  while (!sets.empty() && sets.front() == ' ') sets.erase(0, 1);
  std::vector<PlanItem> items;
  size_t pos = 0;
  while (pos < sets.size()) {
    const size_t e = sets.find(';', pos);
    PlanItem p;
    if (!parse_plan_item(sets.substr(pos, e == std::string::npos ? std::string::npos : e - pos), p)) return false;
    items.push_back(p);
    pos = e == std::string::npos ? sets.size() : e + 1;
  }
  out = items;
  return true;
}

// --- R: one set's result ------------------------------------------------------------------------
inline std::string fmt_result_line(int id, const Result& r) {
  std::string err = r.error;
  for (char& c : err)
    if (c == '\n' || c == '\r') c = ' ';
  const AbftOut& a = r.abft;
  std::string list = a.list.empty() ? "-" : a.list;
  for (char& c : list)
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r') c = '_';
  char buf[1024];
  std::snprintf(buf, sizeof buf,
                "R %d %d %d %d %.17g %.17g %.17g %d %.17g %zu %zu %d %d %d %d %d %d %d %d %d %d %d %d %d %d %d %.17g "
                "%.17g %.17g %.17g %.17g %.17g %.17g ",
                id, r.launched, r.ok, r.oom, r.tflops, r.ms, r.max_rel_err, r.stab_dispatches, r.stab_spread,
                r.need_bytes, r.free_bytes, r.iters, r.ramp, a.ran, a.variant, a.tile_m, a.tile_n, a.bad_tiles, a.tm,
                a.tn, a.wg, a.round, a.xcd, a.se, a.sh, a.cu, a.worst_ratio, a.checked_fraction, a.check_ms, a.abft_ms,
                r.probe_ms, a.dispatch_ms, a.rows_ms);
  return buf + list + " " + err;
}

// One worker result line. False when it does not parse; the error text is whatever follows the
// bad-tile list (possibly empty).
inline bool parse_result_line(const std::string& ln, int& id, Result& out) {
  Result r = out;
  AbftOut& a = r.abft;
  Reader rd{ln};
  std::string tag;
  rd >> tag;
  if (!rd.ok || tag != "R") return false;
  int rid = 0;
  rd >> rid >> r.launched >> r.ok >> r.oom >> r.tflops >> r.ms >> r.max_rel_err >> r.stab_dispatches >> r.stab_spread >>
      r.need_bytes >> r.free_bytes >> r.iters >> r.ramp >> a.ran >> a.variant >> a.tile_m >> a.tile_n >> a.bad_tiles >>
      a.tm >> a.tn >> a.wg >> a.round >> a.xcd >> a.se >> a.sh >> a.cu >> a.worst_ratio >> a.checked_fraction >>
      a.check_ms >> a.abft_ms >> r.probe_ms >> a.dispatch_ms >> a.rows_ms >> a.list;
  if (!rd.ok || a.list.size() > 255) return false;
  size_t p = rd.pos;
  if (p < ln.size() && ln[p] == ' ') ++p;
  r.error = p < ln.size() ? ln.substr(p) : "";
  while (!r.error.empty() && (r.error.back() == '\n' || r.error.back() == '\r')) r.error.pop_back();
  id = rid;
  out = r;
  return true;
}

}  // namespace vproto
