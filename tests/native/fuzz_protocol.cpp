// Random-input loop for amd-gemm-validate's launcher <-> worker line protocol
// (native/include/validate_protocol.h) under AddressSanitizer + UBSan (tests/test_native_sanitizers.py).
// The launcher parses what its worker processes print (S / R lines), the worker what the launcher
// sends (P line, --worker-opts); the command line feeds the shape and index lists.
//   fuzz_protocol [iterations] [seed]
// Properties: no parser crashes on any input; every formatted line parses back to the same fields;
// a line that parses re-formats to a line that parses to the same fields (no half-read result).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "validate_protocol.h"

using namespace vproto;

static uint64_t g_state = 0x243F6A8885A308D3ull;
static uint64_t rnd() {
  uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static int rn(int n) { return (int)(rnd() % (uint64_t)n); }
static int ri() {
  static const int edge[] = {0, 1, -1, 7, 255, 256, 8192, INT32_MAX, INT32_MIN};
  return rn(3) ? rn(100000) - 1000 : edge[rn(9)];
}
static double rd() {
  static const double edge[] = {0.0, -0.0, 1.0, 1e-300, 1e300, 1687.77, 0.1, NAN, INFINITY, -INFINITY};
  return rn(3) ? (double)(rnd() % 1000000) / 1000.0 : edge[rn(10)];
}

static int g_fail = 0;
static void expect(bool ok, const char* what, const std::string& in) {
  if (ok) return;
  std::fprintf(stderr, "FAIL %s: %.300s\n", what, in.c_str());
  ++g_fail;
}
static bool same(double a, double b) { return (std::isnan(a) && std::isnan(b)) || a == b; }

static Result rand_result() {
  Result r;
  r.launched = rn(2), r.ok = rn(2), r.oom = rn(2);
  r.tflops = rd(), r.ms = rd(), r.max_rel_err = rd(), r.stab_spread = rd(), r.probe_ms = rd();
  r.stab_dispatches = ri(), r.iters = ri(), r.ramp = ri();
  r.need_bytes = rnd() >> 2, r.free_bytes = rnd() >> 2;
  AbftOut& a = r.abft;
  a.ran = rn(2), a.variant = ri(), a.tile_m = ri(), a.tile_n = ri(), a.bad_tiles = ri();
  a.tm = ri(), a.tn = ri(), a.wg = ri(), a.round = ri(), a.xcd = ri(), a.se = ri(), a.sh = ri(), a.cu = ri();
  a.worst_ratio = rd(), a.checked_fraction = rd(), a.check_ms = rd(), a.abft_ms = rd();
  a.dispatch_ms = rd(), a.rows_ms = rd();
  a.list = rn(2) ? "-" : std::to_string(rn(99)) + "." + std::to_string(rn(99)) + "." + std::to_string(rn(8) - 1);
  static const char* errs[] = {"", "ABFT: 1 bad tile(s), first [5,7] (workgroup 232, XCD 7)", "gemm launch: x y z",
                               "  leading spaces", "tabs\tand\nnewlines\r", "\xff\xfe binary"};
  r.error = errs[rn(6)];
  return r;
}

static bool equal(const Result& x, const Result& y) {
  const AbftOut &a = x.abft, &b = y.abft;
  return x.launched == y.launched && x.ok == y.ok && x.oom == y.oom && same(x.tflops, y.tflops) && same(x.ms, y.ms) &&
         same(x.max_rel_err, y.max_rel_err) && same(x.stab_spread, y.stab_spread) && same(x.probe_ms, y.probe_ms) &&
         x.stab_dispatches == y.stab_dispatches && x.iters == y.iters && x.ramp == y.ramp &&
         x.need_bytes == y.need_bytes && x.free_bytes == y.free_bytes && a.ran == b.ran && a.variant == b.variant &&
         a.tile_m == b.tile_m && a.tile_n == b.tile_n && a.bad_tiles == b.bad_tiles && a.tm == b.tm && a.tn == b.tn &&
         a.wg == b.wg && a.round == b.round && a.xcd == b.xcd && a.se == b.se && a.sh == b.sh && a.cu == b.cu &&
         same(a.worst_ratio, b.worst_ratio) && same(a.checked_fraction, b.checked_fraction) &&
         same(a.check_ms, b.check_ms) && same(a.abft_ms, b.abft_ms) && same(a.dispatch_ms, b.dispatch_ms) &&
         same(a.rows_ms, b.rows_ms) && a.list == b.list;
}

static std::string mutate(std::string s) {
  static const char alphabet[] = "RSP0123456789-+.eEnaixf :;,\t\n\r\x00\xff";
  for (int m = 1 + rn(4); m > 0; --m) {
    const size_t at = s.empty() ? 0 : (size_t)rn((int)s.size() + 1);
    switch (rn(5)) {
      case 0:
        if (at < s.size()) s[at] = alphabet[rn(sizeof alphabet - 1)];
        break;
      case 1: s.insert(at, 1, alphabet[rn(sizeof alphabet - 1)]); break;
      case 2:
        if (at < s.size()) s.erase(at, 1 + rn(12));
        break;
      case 3: s = s.substr(0, at); break;
      default: s.insert(at, std::string(1 + rn(40), '9'));
    }
  }
  return s;
}

int main(int argc, char** argv) {
  const long iters = argc > 1 ? std::atol(argv[1]) : 20000;
  if (argc > 2) g_state ^= std::strtoull(argv[2], nullptr, 10);
  for (long i = 0; i < iters && g_fail < 20; ++i) {
    // R: round trip, then mutations
    const int id = ri();
    const Result r = rand_result();
    const std::string line = fmt_result_line(id, r);
    int pid = 0;
    Result back;
    expect(parse_result_line(line, pid, back) && pid == id && equal(r, back), "R round trip", line);
    std::string want_err = r.error;
    for (char& c : want_err)
      if (c == '\n' || c == '\r') c = ' ';
    while (!want_err.empty() && want_err.back() == ' ') want_err.pop_back();
    std::string got_err = back.error;
    while (!got_err.empty() && got_err.back() == ' ') got_err.pop_back();
    expect(got_err == want_err, "R error text", line);
    const std::string bad = mutate(line);
    Result m;
    if (parse_result_line(bad, pid, m)) {
      Result again;
      int id2 = 0;
      expect(parse_result_line(fmt_result_line(pid, m), id2, again) && id2 == pid && equal(m, again), "R reparse", bad);
    }
    // S
    const StartLine sl{ri(), rn(2) ? "0000:05:00.0" : "-", rn(2) ? "gfx950:sramecc+:xnack-" : "-", ri(),
                       (size_t)(rnd() >> 4)};
    StartLine sb;
    const std::string sline = fmt_start_line(sl);
    expect(parse_start_line(sline, sb) && sb.ndev == sl.ndev && sb.bus == sl.bus && sb.arch == sl.arch &&
               sb.cus == sl.cus && sb.lds == sl.lds, "S round trip", sline);
    (void)parse_start_line(mutate(sline), sb);
    // P
    std::vector<PlanItem> items;
    std::string pline = "P ";
    for (int k = 1 + rn(6); k > 0; --k) {
      PlanItem p{ri(), rn(2) ? "bf16" : "fp8_e4m3fn", {1 + rn(65536), 1 + rn(65536), 1 + rn(65536)}, 1 + rn(8)};
      items.push_back(p);
      pline += (k == 0 || items.size() == 1 ? "" : ";") + fmt_plan_item(p);
    }
    std::vector<PlanItem> pb;
    bool same_plan = parse_plan_line(pline + "\n", pb) && pb.size() == items.size();
    for (size_t q = 0; same_plan && q < pb.size(); ++q)
      same_plan = pb[q].id == items[q].id && pb[q].dtype == items[q].dtype && pb[q].s.m == items[q].s.m &&
                  pb[q].s.n == items[q].s.n && pb[q].s.k == items[q].s.k && pb[q].set_size == items[q].set_size;
    expect(same_plan, "P round trip", pline);
    const std::string pbad = mutate(pline);
    if (parse_plan_line(pbad, pb))
      for (const auto& p : pb) expect(p.s.m > 0 && p.s.n > 0 && p.s.k > 0 && p.set_size > 0 && !p.dtype.empty(),
                                      "P accepted a bad item", pbad);
    // --worker-opts
    Options o;
    o.iters = ri(), o.warmup = ri(), o.check_rows = ri(), o.stabilise = rn(2), o.inject_tm = ri(), o.inject_tn = ri();
    o.stabilise_max_s = rd(), o.min_window_ms = rd(), o.ramp_ms = rd(), o.pre_idle_ms = rd(), o.inject_delta = rd();
    Options ob;
    const std::string ol = fmt_opts(o);
    expect(parse_opts(ol, ob) && ob.iters == o.iters && ob.warmup == o.warmup && ob.check_rows == o.check_rows &&
               ob.stabilise == o.stabilise && ob.inject_tm == o.inject_tm && ob.inject_tn == o.inject_tn &&
               same(ob.stabilise_max_s, o.stabilise_max_s) && same(ob.inject_delta, o.inject_delta),
           "opts round trip", ol);
    (void)parse_opts(mutate(ol), ob);
    // command-line lists
    std::string spec;
    for (int k = rn(4); k > 0; --k) spec += (spec.empty() ? "" : ",") + std::to_string(ri()) + (rn(2) ? "x7x9" : "");
    std::vector<Shape> shp;
    (void)parse_shapes_strict(mutate(spec), shp);
    std::vector<int> idx;
    (void)parse_index_list(mutate(spec).c_str(), idx);
    (void)parse_ints(mutate(spec));
    // junk
    std::string junk;
    for (int n = rn(200); n > 0; --n) junk += (char)rn(256);
    (void)parse_result_line("R " + junk, pid, m);
    (void)parse_result_line(junk, pid, m);
    (void)parse_plan_line(junk, pb);
    (void)parse_start_line("S " + junk, sb);
    (void)parse_opts(junk, ob);
  }
  // an out-of-range field fails the line instead of wrapping
  int pid = 0;
  Result m;
  std::string over = fmt_result_line(3, Result{});
  over.replace(2, 1, "99999999999999999999");
  expect(!parse_result_line(over, pid, m), "out-of-range id accepted", over);
  std::printf("{\"fuzz\":\"protocol\",\"iterations\":%ld,\"failures\":%d}\n", iters, g_fail);
  return g_fail ? 1 : 0;
}
