// amd-barrier-wait: block an init container until node barrier files appear.
//
//   amd-barrier-wait --dir /run/amd/validations --all toolkit-ready [--timeout 3600]
//   amd-barrier-wait --dir /run/amd/validations --any host-driver-ready,driver-ready
//
// Replaces the reference's `until [ -f /run/nvidia/validations/toolkit-ready ]; do sleep 5;
// done` init containers (e.g. assets/state-device-plugin/0500_daemonset.yaml:31): inotify
// wakes the waiter as the producer writes the file, removing up to 5 s per barrier from
// node time-to-ready. Exit 0 when satisfied, 1 on timeout, 2 on usage error.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "amdnode.h"

static std::vector<std::string> split(const std::string& s) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s + ",") {
    if (c == ',') {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  return out;
}

int main(int argc, char** argv) {
  std::string dir = "/run/amd/validations";
  std::vector<std::string> names;
  bool any = false;
  long long timeout_s = -1;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--dir") dir = next();
    else if (a == "--all") { names = split(next()); any = false; }
    else if (a == "--any") { names = split(next()); any = true; }
    else if (a == "--timeout") timeout_s = std::stoll(next());
    else if (a == "-h" || a == "--help") {
      std::printf("usage: amd-barrier-wait --dir DIR (--all|--any) a,b,... [--timeout SECONDS]\n");
      return 0;
    } else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if (names.empty()) {
    std::fprintf(stderr, "no barrier names given\n");
    return 2;
  }
  auto t0 = std::chrono::steady_clock::now();
  auto have = amdnode::wait_files(dir, names, any, timeout_s < 0 ? -1 : timeout_s * 1000);
  double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (have.empty()) {
    std::fprintf(stderr, "timed out after %.1fs waiting for %s in %s\n", dt, any ? "any barrier" : "all barriers",
                 dir.c_str());
    return 1;
  }
  std::printf("barrier satisfied after %.3fs:", dt);
  for (auto& h : have) std::printf(" %s", h.c_str());
  std::printf("\n");
  return 0;
}
