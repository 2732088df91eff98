// amd-container-runtime: OCI runtime shim that hands AMD GPUs to containers.
//
// Role of the reference's container-toolkit runtime (SURVEY.md §2.3 "container-toolkit"),
// re-designed for ROCm: the amdgpu stack needs no user-space driver libraries injected into
// the container (ROCm ships inside the workload image) — a container only needs the KFD
// node (/dev/kfd) plus the DRM render node(s) of the GPUs it was given, and cgroup device
// access to them. So the shim is small, native and fast (it sits on every container start):
//
//   1. parse runc's command line; anything but `create` is passed straight through;
//   2. load <bundle>/config.json and collect the requested devices from
//        - CDI annotations  (prefix "amd.cdi.k8s.io/", value "amd.com/gpu=0,amd.com/gpu=3"), and
//        - AMD_VISIBLE_DEVICES in the process env ("all", indices, amdgpu-<uid>, PCI BDFs);
//   3. mode cdi:    apply containerEdits of the matching devices from the CDI specs
//                   (/etc/cdi, /var/run/cdi, *.json written by `amd-ctk cdi generate`);
//      mode legacy: resolve devices from the KFD topology (libamdnode) and add /dev/kfd and
//                   /dev/dri/renderD<minor> directly;
//      mode auto:   CDI when a spec for amd.com/gpu exists, else legacy;
//   4. add linux.devices + linux.resources.devices allow rules, write config.json back
//      atomically, and exec the low-level runtime (runc/crun) with the original arguments.
//
// Configuration: <dir of this binary>/amd-container-runtime.conf or
// /etc/amd-container-runtime/config (key = value lines), overridable by environment
// (AMD_CONTAINER_RUNTIME_<KEY>). Keys: mode, runtimes, cdi-spec-dirs, annotation-prefixes,
// sys-root, dev-root, log-file, debug. Invoked as amd-container-runtime.cdi / .legacy (the
// binaries behind the amd-cdi / amd-legacy RuntimeClasses) the mode is pinned.
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/sysmacros.h>
#include <sys/types.h>
#include <unistd.h>
#include <dirent.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "amdnode.h"
#include "minijson.h"

using minijson::Value;

namespace {

struct Config {
  std::string mode = "auto";
  std::vector<std::string> runtimes = {"runc", "crun"};
  std::vector<std::string> cdi_dirs = {"/etc/cdi", "/var/run/cdi"};
  std::vector<std::string> annotation_prefixes = {"amd.cdi.k8s.io/"};
  std::string sys_root = "/";
  std::string dev_root = "/";
  std::string log_file;
  bool debug = false;
};

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n\"'"), b = s.find_last_not_of(" \t\r\n\"'");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, sep)) {
    item = trim(item);
    if (!item.empty()) out.push_back(item);
  }
  return out;
}

FILE* g_log = nullptr;
bool g_debug = false;

void logf(const char* fmt, const std::string& a = "", const std::string& b = "") {
  if (!g_log) return;
  std::fprintf(g_log, "[amd-container-runtime %d] ", int(getpid()));
  std::fprintf(g_log, fmt, a.c_str(), b.c_str());
  std::fputc('\n', g_log);
  std::fflush(g_log);
}

[[noreturn]] void die(const std::string& msg) {
  std::fprintf(stderr, "amd-container-runtime: %s\n", msg.c_str());
  logf("error: %s", msg);
  std::exit(1);
}

void apply_kv(Config& c, const std::string& k, const std::string& v) {
  if (k == "mode") c.mode = v;
  else if (k == "runtimes") c.runtimes = split(v, ',');
  else if (k == "cdi-spec-dirs") c.cdi_dirs = split(v, ':');
  else if (k == "annotation-prefixes") c.annotation_prefixes = split(v, ',');
  else if (k == "sys-root") c.sys_root = v;
  else if (k == "dev-root") c.dev_root = v;
  else if (k == "log-file") c.log_file = v;
  else if (k == "debug") c.debug = (v == "true" || v == "1");
}

std::string self_dir() {
  char buf[4096];
  ssize_t n = readlink("/proc/self/exe", buf, sizeof buf - 1);
  if (n <= 0) return "";
  buf[n] = 0;
  std::string p(buf);
  return p.substr(0, p.rfind('/'));
}

Config load_config() {
  Config c;
  for (const std::string& path : {self_dir() + "/amd-container-runtime.conf",
                                  std::string("/etc/amd-container-runtime/config")}) {
    std::ifstream f(path);
    if (!f) continue;
    std::string line;
    while (std::getline(f, line)) {
      auto hash = line.find('#');
      if (hash != std::string::npos) line.resize(hash);
      auto eq = line.find('=');
      if (eq == std::string::npos) continue;
      apply_kv(c, trim(line.substr(0, eq)), trim(line.substr(eq + 1)));
    }
    break;
  }
  static const char* keys[] = {"mode", "runtimes", "cdi-spec-dirs", "annotation-prefixes", "sys-root",
                               "dev-root", "log-file", "debug"};
  for (const char* k : keys) {
    std::string env = "AMD_CONTAINER_RUNTIME_";
    for (const char* p = k; *p; ++p) env += (*p == '-') ? '_' : char(std::toupper(*p));
    if (const char* v = std::getenv(env.c_str())) apply_kv(c, k, v);
  }
  return c;
}

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

void write_atomic(const std::string& path, const std::string& data) {
  std::string tmp = path + ".amd-tmp";
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
  if (fd < 0) die("cannot write " + tmp + ": " + std::strerror(errno));
  size_t off = 0;
  while (off < data.size()) {
    ssize_t n = ::write(fd, data.data() + off, data.size() - off);
    if (n < 0) { if (errno == EINTR) continue; ::close(fd); die("write failed: " + std::string(std::strerror(errno))); }
    off += size_t(n);
  }
  ::fsync(fd);
  ::close(fd);
  if (::rename(tmp.c_str(), path.c_str()) != 0) die("rename failed: " + std::string(std::strerror(errno)));
}

// ---- command line --------------------------------------------------------------------------
// runc global flags that take a value (the subcommand is the first other non-flag argument)
const std::set<std::string> kGlobalWithValue = {"--root", "--log", "--log-format", "--criu", "--rootless"};

struct Cmd {
  std::string sub;
  std::string bundle = ".";
};

Cmd parse_cmd(int argc, char** argv) {
  Cmd c;
  int i = 1;
  for (; i < argc; ++i) {
    std::string a = argv[i];
    if (a.empty() || a[0] != '-') { c.sub = a; ++i; break; }
    if (a.find('=') == std::string::npos && kGlobalWithValue.count(a)) ++i;
  }
  for (; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--bundle" || a == "-b") { if (i + 1 < argc) c.bundle = argv[++i]; }
    else if (a.rfind("--bundle=", 0) == 0) c.bundle = a.substr(9);
    else if (a.rfind("-b=", 0) == 0) c.bundle = a.substr(3);
  }
  return c;
}

// ---- device requests ------------------------------------------------------------------------
struct Request {
  std::vector<std::string> cdi;      // fully-qualified CDI names (vendor/class=name)
  std::vector<std::string> env;      // raw AMD_VISIBLE_DEVICES entries
};

Request collect_requests(const Value& spec, const Config& cfg) {
  Request r;
  if (const Value* ann = spec.find("annotations"); ann && ann->is_object()) {
    for (auto& kv : ann->o)
      for (auto& pre : cfg.annotation_prefixes)
        if (kv.first.rfind(pre, 0) == 0)
          for (auto& n : split(kv.second.str(), ',')) r.cdi.push_back(n);
  }
  if (const Value* proc = spec.find("process"))
    if (const Value* env = proc->find("env"); env && env->is_array())
      for (auto& e : env->a) {
        const std::string& s = e.s;
        if (s.rfind("AMD_VISIBLE_DEVICES=", 0) == 0) {
          std::string v = s.substr(20);
          r.env = (v == "none" || v == "void" || v.empty()) ? std::vector<std::string>{} : split(v, ',');
        }
      }
  return r;
}

// ---- device nodes ---------------------------------------------------------------------------
struct DevNode {
  std::string path;       // in the container
  std::string host_path;  // on the host
  std::string type = "c";
  long long major = -1, minor = -1;
  std::string permissions = "rwm";
  long long file_mode = 0666;
};

void stat_node(DevNode& d, const Config& cfg) {
  if (d.major >= 0 && d.minor >= 0) return;
  std::string hp = amdnode::join(cfg.dev_root, d.host_path.empty() ? d.path : d.host_path);
  struct stat st;
  if (::stat(hp.c_str(), &st) != 0) die("device node " + hp + " missing: " + std::strerror(errno));
  if (S_ISCHR(st.st_mode)) d.type = "c";
  else if (S_ISBLK(st.st_mode)) d.type = "b";
  else die(hp + " is not a device node");
  d.major = major(st.st_rdev);
  d.minor = minor(st.st_rdev);
}

struct Edits {
  std::vector<DevNode> nodes;
  std::vector<std::string> env;
  std::vector<Value> mounts;
  std::vector<std::pair<std::string, Value>> hooks;   // hook name -> hook object
};

void merge_edits(Edits& e, const Value* ce) {
  if (!ce || !ce->is_object()) return;
  if (const Value* env = ce->find("env"); env && env->is_array())
    for (auto& v : env->a) e.env.push_back(v.s);
  if (const Value* dn = ce->find("deviceNodes"); dn && dn->is_array())
    for (auto& v : dn->a) {
      DevNode d;
      if (const Value* x = v.find("path")) d.path = x->s;
      if (const Value* x = v.find("hostPath")) d.host_path = x->s;
      if (const Value* x = v.find("type")) d.type = x->s;
      if (const Value* x = v.find("major")) d.major = x->integer(-1);
      if (const Value* x = v.find("minor")) d.minor = x->integer(-1);
      if (const Value* x = v.find("permissions")) d.permissions = x->s;
      if (const Value* x = v.find("fileMode")) d.file_mode = x->integer(0666);
      e.nodes.push_back(d);
    }
  if (const Value* m = ce->find("mounts"); m && m->is_array())
    for (auto& v : m->a) e.mounts.push_back(v);
  if (const Value* h = ce->find("hooks"); h && h->is_array())
    for (auto& v : h->a) {
      Value hook = Value::object();
      std::string name = v.find("hookName") ? v.find("hookName")->s : "createContainer";
      for (auto& kv : v.o) if (kv.first != "hookName") hook[kv.first] = kv.second;
      e.hooks.emplace_back(name, hook);
    }
}

// CDI registry: kind "amd.com/gpu" -> name -> containerEdits (plus spec-wide edits)
struct CdiSpec {
  Value doc;
  const Value* common = nullptr;
  std::map<std::string, const Value*> devices;
};

std::vector<CdiSpec> load_cdi(const Config& cfg, const std::string& kind) {
  std::vector<CdiSpec> out;
  for (auto& dir : cfg.cdi_dirs) {
    DIR* d = ::opendir(dir.c_str());
    if (!d) continue;
    std::vector<std::string> files;
    while (dirent* de = ::readdir(d)) {
      std::string n = de->d_name;
      if (n.size() > 5 && n.compare(n.size() - 5, 5, ".json") == 0) files.push_back(dir + "/" + n);
    }
    ::closedir(d);
    std::sort(files.begin(), files.end());
    for (auto& f : files) {
      std::string text;
      if (!read_file(f, text)) continue;
      CdiSpec s;
      try {
        s.doc = minijson::parse(text);
      } catch (const std::exception& e) {
        logf("skipping CDI spec %s: %s", f, e.what());
        continue;
      }
      if (!s.doc.find("kind") || s.doc.find("kind")->s != kind) continue;
      out.push_back(std::move(s));
    }
  }
  for (auto& s : out) {   // pointers into s.doc are stable now that the vector is final
    s.common = s.doc.find("containerEdits");
    if (const Value* devs = s.doc.find("devices"); devs && devs->is_array())
      for (auto& dv : devs->a)
        if (const Value* n = dv.find("name")) s.devices[n->s] = dv.find("containerEdits");
  }
  return out;
}

bool resolve_cdi(const std::vector<std::string>& names, const Config& cfg, Edits& e, std::string& err) {
  std::map<std::string, std::vector<std::string>> by_kind;
  for (auto& n : names) {
    auto eq = n.find('=');
    if (eq == std::string::npos) { err = "invalid CDI device name " + n; return false; }
    by_kind[n.substr(0, eq)].push_back(n.substr(eq + 1));
  }
  for (auto& [kind, devs] : by_kind) {
    auto specs = load_cdi(cfg, kind);
    std::set<const Value*> commons;
    for (auto& dn : devs) {
      bool found = false;
      for (auto& s : specs) {
        auto it = s.devices.find(dn);
        if (it == s.devices.end()) continue;
        merge_edits(e, it->second);
        if (s.common && commons.insert(s.common).second) merge_edits(e, s.common);
        found = true;
        break;
      }
      if (!found) { err = "unresolvable CDI device " + kind + "=" + dn; return false; }
    }
  }
  return true;
}

bool have_cdi_kind(const Config& cfg, const std::string& kind) { return !load_cdi(cfg, kind).empty(); }

// Legacy: map AMD_VISIBLE_DEVICES entries to KFD agents directly.
void resolve_legacy(const std::vector<std::string>& req, const Config& cfg, Edits& e) {
  auto gpus = amdnode::enumerate_gpus(cfg.sys_root);
  std::vector<const amdnode::Gpu*> sel;
  auto add = [&](const amdnode::Gpu* g) {
    if (std::find(sel.begin(), sel.end(), g) == sel.end()) sel.push_back(g);
  };
  for (auto& r : req) {
    if (r == "all") { for (auto& g : gpus) add(&g); continue; }
    bool ok = false;
    for (auto& g : gpus) {
      char uid[40];
      std::snprintf(uid, sizeof uid, "%016llx", (unsigned long long)g.unique_id);
      std::string id = r;
      if (id.rfind("amdgpu-", 0) == 0) id = id.substr(7);
      else if (id.rfind("GPU-", 0) == 0) id = id.substr(4);
      bool is_index = !r.empty() && std::all_of(r.begin(), r.end(), ::isdigit);
      if ((is_index && std::stoi(r) == g.index) || id == uid || r == g.pci_bdf) { add(&g); ok = true; }
    }
    if (!ok) die("AMD_VISIBLE_DEVICES entry " + r + " matches no GPU");
  }
  if (sel.empty()) return;
  DevNode kfd;
  kfd.path = "/dev/kfd";
  e.nodes.push_back(kfd);
  for (auto* g : sel) {
    if (g->drm_render_minor < 0) continue;
    DevNode d;
    d.path = "/dev/dri/renderD" + std::to_string(g->drm_render_minor);
    e.nodes.push_back(d);
  }
}

// ---- spec edits -----------------------------------------------------------------------------
void apply(Value& spec, Edits& e, const Config& cfg) {
  // Objects are vectors of members: create every key first, then take references (a later
  // insertion into the same object would reallocate and dangle an earlier reference).
  Value& linux_ = spec["linux"];
  linux_["devices"];
  linux_["resources"]["devices"];
  Value& devs = *linux_.find("devices");
  if (devs.is_null()) devs = Value::array();
  Value& allow = (*linux_.find("resources"))["devices"];
  if (allow.is_null()) allow = Value::array();
  std::set<std::string> have;
  for (auto& d : devs.a) if (const Value* p = d.find("path")) have.insert(p->s);
  for (auto& n : e.nodes) {
    stat_node(n, cfg);
    if (have.insert(n.path).second) {
      Value d = Value::object();
      d["path"] = Value::string(n.path);
      d["type"] = Value::string(n.type);
      d["major"] = Value::number(n.major);
      d["minor"] = Value::number(n.minor);
      d["fileMode"] = Value::number(n.file_mode);
      d["uid"] = Value::number(0);
      d["gid"] = Value::number(0);
      devs.push(d);
    }
    Value rule = Value::object();
    rule["allow"] = Value::boolean(true);
    rule["type"] = Value::string(n.type);
    rule["major"] = Value::number(n.major);
    rule["minor"] = Value::number(n.minor);
    rule["access"] = Value::string(n.permissions);
    allow.push(rule);
    logf("inject %s", n.path);
  }
  if (!e.env.empty()) {
    Value& env = spec["process"]["env"];
    if (env.is_null()) env = Value::array();
    for (auto& kv : e.env) {
      std::string key = kv.substr(0, kv.find('='));
      auto it = std::find_if(env.a.begin(), env.a.end(),
                             [&](const Value& v) { return v.s.rfind(key + "=", 0) == 0; });
      if (it != env.a.end()) it->s = kv;
      else env.push(Value::string(kv));
    }
  }
  if (!e.mounts.empty()) {
    Value& mounts = spec["mounts"];
    if (mounts.is_null()) mounts = Value::array();
    for (auto& m : e.mounts) {
      Value mm = Value::object();
      if (const Value* x = m.find("containerPath")) mm["destination"] = *x;
      if (const Value* x = m.find("hostPath")) mm["source"] = *x;
      mm["type"] = m.find("type") ? *m.find("type") : Value::string("bind");
      mm["options"] = m.find("options") ? *m.find("options") : Value::array();
      if (mm["options"].a.empty()) { mm["options"].push(Value::string("rbind")); mm["options"].push(Value::string("ro")); }
      mounts.push(mm);
    }
  }
  for (auto& [name, hook] : e.hooks) {
    Value& list = spec["hooks"][name];
    if (list.is_null()) list = Value::array();
    list.push(hook);
  }
}

std::string find_runtime(const Config& cfg) {
  for (auto& r : cfg.runtimes) {
    if (r.find('/') != std::string::npos) {
      if (::access(r.c_str(), X_OK) == 0) return r;
      continue;
    }
    const char* path = std::getenv("PATH");
    std::string p = path ? path : "/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin";
    for (auto& dir : split(p, ':')) {
      std::string cand = dir + "/" + r;
      if (::access(cand.c_str(), X_OK) == 0) return cand;
    }
  }
  die("no low-level OCI runtime found (tried " + std::to_string(cfg.runtimes.size()) + " candidates)");
}

int modify_bundle(const std::string& bundle, const Config& cfg) {
  std::string path = bundle + "/config.json";
  std::string text;
  if (!read_file(path, text)) die("cannot read " + path);
  Value spec;
  try {
    spec = minijson::parse(text);
  } catch (const std::exception& ex) {
    die(std::string("invalid ") + path + ": " + ex.what());
  }
  Request req = collect_requests(spec, cfg);
  if (req.cdi.empty() && req.env.empty()) return 0;   // not a GPU container: untouched
  Edits e;
  std::string mode = cfg.mode;
  if (mode == "auto") mode = have_cdi_kind(cfg, "amd.com/gpu") ? "cdi" : "legacy";
  std::vector<std::string> cdi_names = req.cdi;
  if (mode == "cdi") {
    for (auto& r : req.env) cdi_names.push_back(r.find('=') == std::string::npos ? "amd.com/gpu=" + r : r);
  } else if (!req.env.empty()) {
    resolve_legacy(req.env, cfg, e);
  }
  if (!cdi_names.empty()) {
    std::string err;
    if (!resolve_cdi(cdi_names, cfg, e, err)) die(err);
  }
  apply(spec, e, cfg);
  write_atomic(path, minijson::dump(spec));
  logf("bundle %s: %s", bundle, std::to_string(e.nodes.size()) + " device node(s), mode " + mode);
  return int(e.nodes.size());
}

}  // namespace

int main(int argc, char** argv) {
  auto t0 = std::chrono::steady_clock::now();
  Config cfg = load_config();
  // mode-pinned entry points installed as symlinks: amd-container-runtime.cdi / .legacy
  std::string self = argv[0];
  for (const char* m : {"cdi", "legacy"}) {
    std::string suffix = std::string(".") + m;
    if (self.size() > suffix.size() && self.compare(self.size() - suffix.size(), suffix.size(), suffix) == 0)
      cfg.mode = m;
  }
  g_debug = cfg.debug;
  if (!cfg.log_file.empty()) g_log = std::fopen(cfg.log_file.c_str(), "a");
  Cmd cmd = parse_cmd(argc, argv);
  if (cmd.sub == "create") modify_bundle(cmd.bundle, cfg);
  std::string rt = find_runtime(cfg);
  if (g_log) {
    auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    logf("exec %s (%s us in shim)", rt, std::to_string(us));
    std::fclose(g_log);
  }
  std::vector<char*> args;
  args.push_back(const_cast<char*>(rt.c_str()));
  for (int i = 1; i < argc; ++i) args.push_back(argv[i]);
  args.push_back(nullptr);
  ::execv(rt.c_str(), args.data());
  std::fprintf(stderr, "amd-container-runtime: exec %s: %s\n", rt.c_str(), std::strerror(errno));
  return 127;
}
