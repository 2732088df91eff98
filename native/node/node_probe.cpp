// amd-node-probe: print the node's AMD GPU topology and driver state as JSON.
//   amd-node-probe [--root /host] [--dev-root /]
#include <cstdio>
#include <string>

#include "amdnode.h"

int main(int argc, char** argv) {
  std::string root = "/", dev_root = "/";
  for (int i = 1; i + 1 < argc; ++i) {
    std::string a = argv[i];
    if (a == "--root") root = argv[++i];
    else if (a == "--dev-root") dev_root = argv[++i];
  }
  auto gpus = amdnode::enumerate_gpus(root);
  auto drv = amdnode::driver_state(root, dev_root);
  std::printf("%s\n", amdnode::to_json(gpus, drv).c_str());
  return 0;
}
