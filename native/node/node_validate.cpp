// amd-node-validate: the validator components that need no Kubernetes API, as one static binary.
//
//   amd-node-validate driver  [--with-wait] [--output-dir DIR] [--wait-timeout S]
//   amd-node-validate toolkit [--with-wait] [--output-dir DIR] [--wait-timeout S]
//   amd-node-validate rccl    [--output-dir DIR]
//   amd-node-validate plugin  [--output-dir DIR]
//
// The same checks and barrier payloads as validator/components.py (validate_driver,
// validate_toolkit, the no-fabric branch of validate_rccl), without a Python interpreter on the
// node bring-up's critical path: each of these init containers starts, checks sysfs and writes its
// barrier in milliseconds (reference: validator/main.go:607-679 driver, :775-801 toolkit). The
// components that talk to the API server (hip, plugin, the fabric pod) stay in `amd-validator`.
//
// plugin (WITH_WORKLOAD=false, the DaemonSet's setting): GETs this Node, then watches it (one watch,
// fieldSelector=metadata.name, on the same kept-alive connection), bounded by 150 s like the
// validator's event-driven wait, until its capacity advertises amd.com/gpu (or,
// PARTITION_STRATEGY=mixed, amd.com/partition-*), then writes plugin-ready -- one connection and one
// TLS handshake per node, not a request every 100 ms. The API server is reached in-cluster
// (service-account token and CA, TLS through OpenSSL with host-name verification) or through the
// current context of a KUBECONFIG whose user has a token or no credentials. Anything else -- a
// workload pod to spawn, client certificates, the reference's poll mode, an unreachable API -- exits 3
// and `amd-validator` does it.
//
// rccl: a node with fewer than 2 physical GPUs (KFD agents grouped by PCI function) has no fabric;
// rccl-ready is written with a skip. With 2 or more (or none enumerated, where the validator reads
// the node's labels) it exits 3 without writing anything: the init container then execs
// `amd-validator`, which plans and runs the fabric pod.
//
// Environment (the validator's names): WITH_WAIT, OUTPUT_DIR, WAIT_TIMEOUT_SECONDS,
// SLEEP_INTERVAL_SECONDS, AMD_SYSFS_ROOT, AMD_DEV_ROOT, HOST_ROOT, DRIVER_ROOT_MODE (host |
// container), DRIVER_VALIDATION_STRICT, AMD_MOUNTS (process-level node harnesses: container path ->
// host path pairs, utils/mounts.py). Exit 0 ok, 1 validation failed, 2 usage, 3 not handled here.
//
// A barrier that already exists with the same name keeps its first `ts` (when the layer was first
// found ready -- the start of node time-to-ready) and gets `revalidated_ts`: a validator restart
// re-checks the driver without moving the moment it became ready.
#include <arpa/inet.h>
#include <netdb.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "amdnode.h"
#include "minijson.h"

namespace {

using minijson::Value;

std::string env(const char* k, const std::string& dflt = "") {
  const char* v = std::getenv(k);
  return v ? std::string(v) : dflt;
}

bool truthy(const std::string& v) {
  std::string s = v;
  std::transform(s.begin(), s.end(), s.begin(), ::tolower);
  return s == "1" || s == "true" || s == "yes" || s == "on";
}

bool exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

// utils/mounts.py: AMD_MOUNTS maps container paths to where this process finds them; unset in a
// real container (identity).
std::string mount_path(const std::string& p) {
  static std::vector<std::pair<std::string, std::string>> pairs = [] {
    std::vector<std::pair<std::string, std::string>> out;
    const std::string raw = env("AMD_MOUNTS");
    if (raw.empty()) return out;
    try {
      const Value v = minijson::parse(raw);
      for (const auto& pr : v.a) {
        if (pr.a.size() != 2) continue;
        std::string c = pr.a[0].str();
        while (c.size() > 1 && c.back() == '/') c.pop_back();
        if (c.empty() || c[0] != '/') c = "/" + c;
        out.emplace_back(c, pr.a[1].str());
      }
    } catch (const std::exception&) {
    }
    std::stable_sort(out.begin(), out.end(), [](const auto& a, const auto& b) { return a.first.size() > b.first.size(); });
    return out;
  }();
  if (p.empty() || p[0] != '/') return p;
  for (const auto& [c, h] : pairs) {
    if (c == "/") return p == "/" ? h : (h.back() == '/' ? h : h + "/") + p.substr(1);
    if (p == c) return h;
    if (p.compare(0, c.size() + 1, c + "/") == 0) {
      std::string base = h;
      while (base.size() > 1 && base.back() == '/') base.pop_back();
      return base + p.substr(c.size());
    }
  }
  return p;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

std::string num(double v) {
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.6f", v);
  return buf;
}

Value strings(const std::set<std::string>& xs) {
  Value a = Value::array();
  for (const auto& x : xs) a.push(Value::string(x));
  return a;
}

class ValidationError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

struct Opts {
  std::string component, out_dir, sys_root, dev_root, host_root;
  bool with_wait = false;
  double wait_timeout = 3600, sleep_interval = 5;
};

// Atomic barrier write (tmp + rename, like validator/status.py), keeping an existing barrier's `ts`.
void write_barrier(const Opts& o, const std::string& name, Value info) {
  ::mkdir(o.out_dir.c_str(), 0755);
  const std::string path = o.out_dir + "/" + name;
  const double t = now_s();
  std::string first;
  {
    std::ifstream f(path);
    if (f) {
      std::stringstream ss;
      ss << f.rdbuf();
      try {
        const Value old = minijson::parse(ss.str());
        if (const Value* ts = old.find("ts"); ts && ts->kind == Value::Number) first = ts->s;
      } catch (const std::exception&) {
      }
    }
  }
  if (!first.empty()) {
    info["ts"] = Value::number_text(first);
    info["revalidated_ts"] = Value::number_text(num(t));
  } else {
    info["ts"] = Value::number_text(num(t));
  }
  info["validator"] = Value::string("native");
  const std::string tmp = o.out_dir + "/." + name + ".tmp." + std::to_string(::getpid());
  {
    std::ofstream f(tmp);
    f << minijson::dump(info);
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw ValidationError("cannot write barrier " + path);
}

void remove_barrier(const Opts& o, const std::string& name) { ::unlink((o.out_dir + "/" + name).c_str()); }

// retry() of components.py: once, or (with-wait) until the check passes or the wait is over.
template <typename F>
Value retry(const Opts& o, const char* what, F check) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(o.wait_timeout);
  double delay = 0.2;
  for (;;) {
    try {
      return check();
    } catch (const ValidationError& e) {
      if (!o.with_wait || std::chrono::steady_clock::now() >= deadline) throw;
      std::fprintf(stderr, "%s not ready (%s); retrying in %.1fs\n", what, e.what(), delay);
      std::this_thread::sleep_for(std::chrono::duration<double>(delay));
      delay = std::min(o.sleep_interval, delay * 2);
    }
  }
}

// --- driver (components.validate_driver) ----------------------------------------------------
bool host_driver_installed(const Opts& o) {
  const std::string mode = env("DRIVER_ROOT_MODE");
  if (!mode.empty()) return mode == "host";
  for (const char* m : {"/usr/bin/amd-smi", "/opt/rocm/bin/amd-smi", "/usr/sbin/amdgpu-install"})
    if (exists(o.host_root + m)) return true;
  return false;
}

Value check_driver(const Opts& o) {
  const auto st = amdnode::driver_state(o.sys_root, o.dev_root);
  if (!st.module_loaded) throw ValidationError("amdgpu module not loaded");
  if (!st.live) throw ValidationError("amdgpu initstate is not live");
  if (!st.kfd_present) throw ValidationError("/dev/kfd missing");
  if (st.kfd_gpu_nodes == 0) throw ValidationError("KFD reports no GPU agents");
  const auto gpus = amdnode::enumerate_gpus(o.sys_root);
  std::set<std::string> bound, gfx, products;
  for (const auto& g : gpus) {
    bound.insert(g.pci_bdf);
    gfx.insert(g.gfx_target);
    if (!g.product_name.empty()) products.insert(g.product_name);
  }
  std::vector<std::string> missing;
  for (const auto& f : amdnode::scan_pci(o.sys_root))
    if (!f.is_virtfn && f.driver == "amdgpu" && !bound.count(f.bdf)) missing.push_back(f.bdf);
  if (!missing.empty() && env("DRIVER_VALIDATION_STRICT", "true") == "true") {
    std::string m;
    for (const auto& b : missing) m += (m.empty() ? "" : ", ") + b;
    throw ValidationError("amdgpu-bound GPUs without a KFD agent: [" + m + "]");
  }
  Value info = Value::object();
  info["driver_version"] = Value::string(st.version.empty() ? "inbox" : st.version);
  info["gpus"] = Value::number((long long)bound.size());
  info["kfd_agents"] = Value::number(st.kfd_gpu_nodes);
  info["gfx"] = strings(gfx);
  info["hidden_gpus"] = Value::number((long long)missing.size());
  info["products"] = strings(products);
  return info;
}

Value validate_driver(const Opts& o) {
  const bool host = host_driver_installed(o);
  if (!host && !exists(o.out_dir + "/.driver-ctr-ready")) {
    // the driver container's startup probe writes .driver-ctr-ready once amdgpu is live
    if (!o.with_wait) throw ValidationError("driver container not ready (.driver-ctr-ready missing)");
    if (amdnode::wait_files(o.out_dir, {".driver-ctr-ready"}, false, (int64_t)(o.wait_timeout * 1000)).empty())
      throw ValidationError("timed out waiting for the driver container");
  }
  Value info = retry(o, "driver", [&] { return check_driver(o); });
  info["mode"] = Value::string(host ? "host" : "container");
  const std::string name = host ? "host-driver-ready" : "driver-ready";
  remove_barrier(o, host ? "driver-ready" : "host-driver-ready");
  write_barrier(o, name, info);
  return info;
}

// --- toolkit (components.validate_toolkit) --------------------------------------------------
Value check_toolkit(const Opts& o) {
  if (!exists(amdnode::join(o.dev_root, "/dev/kfd"))) throw ValidationError("/dev/kfd not injected into the container");
  std::set<std::string> render;
  if (DIR* d = ::opendir(amdnode::join(o.dev_root, "/dev/dri").c_str())) {
    while (dirent* e = ::readdir(d))
      if (std::strncmp(e->d_name, "renderD", 7) == 0) render.insert(e->d_name);
    ::closedir(d);
  }
  std::set<std::string> missing;
  for (const auto& g : amdnode::enumerate_gpus(o.sys_root))
    if (g.drm_render_minor >= 0 && !render.count("renderD" + std::to_string(g.drm_render_minor)))
      missing.insert("renderD" + std::to_string(g.drm_render_minor));
  if (!missing.empty()) {
    std::string m;
    for (const auto& x : missing) m += (m.empty() ? "'" : ", '") + x + "'";
    throw ValidationError("render nodes not injected: [" + m + "]");
  }
  Value info = Value::object();
  info["render_nodes"] = Value::number((long long)render.size());
  info["kfd"] = Value::boolean(true);
  return info;
}

Value validate_toolkit(const Opts& o) {
  Value info = retry(o, "toolkit", [&] { return check_toolkit(o); });
  write_barrier(o, "toolkit-ready", info);
  return info;
}

constexpr int kNotHandled = 3;

// Exit 3: a case only the Python validator handles (see the header).
class NotHandled : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// --- a minimal Kubernetes API GET (plugin) --------------------------------------------------
struct Api {
  std::string host, prefix, token, ca_file, ca_pem;
  int port = 443;
  bool tls = true, verify = true;
};

std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

std::string trim(std::string s) {
  const auto b = s.find_first_not_of(" \t\r\n\"'");
  const auto e = s.find_last_not_of(" \t\r\n\"'");
  return b == std::string::npos ? "" : s.substr(b, e - b + 1);
}

void parse_url(const std::string& url, Api& a) {
  std::string rest = url;
  if (rest.rfind("https://", 0) == 0) {
    a.tls = true;
    rest = rest.substr(8);
  } else if (rest.rfind("http://", 0) == 0) {
    a.tls = false;
    rest = rest.substr(7);
  } else {
    throw NotHandled("API server URL " + url);
  }
  const auto slash = rest.find('/');
  std::string hostport = rest.substr(0, slash);
  a.prefix = slash == std::string::npos ? "" : rest.substr(slash);
  while (!a.prefix.empty() && a.prefix.back() == '/') a.prefix.pop_back();
  a.port = a.tls ? 443 : 80;
  if (!hostport.empty() && hostport[0] == '[') {              // [v6]:port
    const auto rb = hostport.find(']');
    a.host = hostport.substr(1, rb - 1);
    if (rb + 1 < hostport.size() && hostport[rb + 1] == ':') a.port = std::atoi(hostport.c_str() + rb + 2);
  } else {
    const auto colon = hostport.rfind(':');
    a.host = colon == std::string::npos ? hostport : hostport.substr(0, colon);
    if (colon != std::string::npos) a.port = std::atoi(hostport.c_str() + colon + 1);
  }
}

std::string b64decode(const std::string& in) {
  static const std::string chars = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  int val = 0, bits = -8;
  for (char c : in) {
    const auto p = chars.find(c);
    if (p == std::string::npos) continue;
    val = (val << 6) + (int)p;
    bits += 6;
    if (bits >= 0) {
      out.push_back((char)((val >> bits) & 0xFF));
      bits -= 8;
    }
  }
  return out;
}

// A KUBECONFIG, block-style YAML only: its `clusters`, `contexts` and `users` lists as name -> fields
// (a list item's nested keys flattened: cluster.server -> server, user.token -> token) and
// `current-context`. Flow style or anything else this reader cannot follow is NotHandled.
struct KubeConfig {
  std::vector<std::map<std::string, std::string>> clusters, contexts, users;
  std::string current;
};

KubeConfig parse_kubeconfig(const std::string& text) {
  KubeConfig kc;
  std::istringstream in(text);
  std::string line;
  std::vector<std::map<std::string, std::string>>* section = nullptr;
  while (std::getline(in, line)) {
    const auto hash = line.find(" #");
    if (hash != std::string::npos) line = line.substr(0, hash);
    if (!line.empty() && line[0] == '#') continue;
    const size_t indent = line.find_first_not_of(' ');
    if (indent == std::string::npos) continue;
    std::string t = line.substr(indent);
    while (!t.empty() && (t.back() == '\r' || t.back() == ' ')) t.pop_back();
    if (t.empty()) continue;
    if (t.find('{') != std::string::npos || t.find('[') == 0) throw NotHandled("kubeconfig in YAML flow style");
    const auto colon = t.find(':');
    if (indent == 0 && t.rfind("- ", 0) != 0 && t != "-") {    // a top-level key (list items may sit at 0)
      const std::string key = t.substr(0, colon);
      section = key == "clusters" ? &kc.clusters : key == "contexts" ? &kc.contexts : key == "users" ? &kc.users : nullptr;
      if (key == "current-context" && colon != std::string::npos) kc.current = trim(t.substr(colon + 1));
      continue;
    }
    if (!section) continue;
    if (t.rfind("- ", 0) == 0 || t == "-") {
      section->emplace_back();
      t = t.size() > 2 ? trim(t.substr(2)) : "";
      if (t.empty()) continue;
    }
    if (section->empty()) throw NotHandled("kubeconfig list without items");
    const auto c = t.find(':');
    if (c == std::string::npos) continue;
    const std::string key = t.substr(0, c), value = trim(t.substr(c + 1));
    if (!value.empty()) section->back()[key] = value;
    else if (key != "cluster" && key != "user" && key != "context") section->back()[key] = "";
  }
  return kc;
}

// In-cluster (service account), or the current context of a KUBECONFIG whose user authenticates
// with a token or not at all; else NotHandled.
Api api_config() {
  Api a;
  const std::string sa = mount_path("/var/run/secrets/kubernetes.io/serviceaccount");
  const std::string host = env("KUBERNETES_SERVICE_HOST");
  if (!host.empty() && exists(sa + "/token")) {
    a.host = host;
    a.port = std::atoi(env("KUBERNETES_SERVICE_PORT", "443").c_str());
    a.tls = true;
    a.token = trim(slurp(sa + "/token"));
    a.ca_file = sa + "/ca.crt";
    return a;
  }
  const std::string path = env("KUBECONFIG");
  if (path.empty() || !exists(path)) throw NotHandled("no in-cluster service account and no KUBECONFIG");
  const KubeConfig kc = parse_kubeconfig(slurp(path));
  auto by_name = [](const std::vector<std::map<std::string, std::string>>& v, const std::string& name,
                    const char* what) -> const std::map<std::string, std::string>* {
    const std::map<std::string, std::string>* hit = nullptr;
    for (const auto& m : v) {
      const auto n = m.find("name");
      if (n != m.end() && n->second == name) {
        if (hit) throw NotHandled(std::string("kubeconfig: two ") + what + " named " + name);
        hit = &m;
      }
    }
    return hit;
  };
  // the context: current-context, or the only one; none at all: the only cluster and user
  const std::map<std::string, std::string>* ctx = nullptr;
  if (!kc.current.empty()) {
    ctx = by_name(kc.contexts, kc.current, "contexts");
    if (!ctx) throw NotHandled("kubeconfig: current-context " + kc.current + " not found");
  } else if (kc.contexts.size() == 1) {
    ctx = &kc.contexts[0];
  } else if (!kc.contexts.empty()) {
    throw NotHandled("kubeconfig: several contexts and no current-context");
  }
  const std::map<std::string, std::string>* cluster = nullptr;
  const std::map<std::string, std::string>* user = nullptr;
  if (ctx) {
    const auto cn = ctx->find("cluster");
    if (cn == ctx->end()) throw NotHandled("kubeconfig: context without a cluster");
    cluster = by_name(kc.clusters, cn->second, "clusters");
    const auto un = ctx->find("user");
    if (un != ctx->end()) {
      user = by_name(kc.users, un->second, "users");
      if (!user) throw NotHandled("kubeconfig: user " + un->second + " not found");
    }
  } else {
    if (kc.clusters.size() != 1 || kc.users.size() > 1) throw NotHandled("kubeconfig without a context to select by");
    cluster = &kc.clusters[0];
    user = kc.users.empty() ? nullptr : &kc.users[0];
  }
  if (!cluster || !cluster->count("server")) throw NotHandled("kubeconfig: the context's cluster has no server");
  auto get = [](const std::map<std::string, std::string>* m, const char* k) {
    if (!m) return std::string();
    const auto it = m->find(k);
    return it == m->end() ? std::string() : it->second;
  };
  if (user)
    for (const char* k : {"client-certificate", "client-certificate-data", "client-key", "client-key-data", "exec",
                          "auth-provider", "tokenFile", "username", "password"})
      if (user->count(k)) throw NotHandled(std::string("kubeconfig user credentials: ") + k);
  a.token = get(user, "token");
  a.ca_file = get(cluster, "certificate-authority");
  const std::string ca_data = get(cluster, "certificate-authority-data");
  if (!ca_data.empty()) a.ca_pem = b64decode(ca_data);
  a.verify = get(cluster, "insecure-skip-tls-verify") != "true";
  parse_url(get(cluster, "server"), a);
  return a;
}

// One connection to the API server (TLS through OpenSSL with host-name verification), buffered,
// kept alive across requests. Transport problems are NotHandled: the Python validator then retries
// and reports them properly.
class Conn {
 public:
  Conn(const Api& a, double timeout_s) : a_(a) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(a.host.c_str(), std::to_string(a.port).c_str(), &hints, &res) != 0 || !res)
      throw NotHandled("cannot resolve " + a.host);
    for (addrinfo* r = res; r && fd_ < 0; r = r->ai_next) {
      fd_ = ::socket(r->ai_family, r->ai_socktype, r->ai_protocol);
      if (fd_ < 0) continue;
      set_timeout(timeout_s);
      if (::connect(fd_, r->ai_addr, r->ai_addrlen) != 0) {
        ::close(fd_);
        fd_ = -1;
      }
    }
    freeaddrinfo(res);
    if (fd_ < 0) throw NotHandled("cannot connect to " + a.host + ":" + std::to_string(a.port));
    if (a.tls) handshake();
  }
  ~Conn() {
    if (ssl_) SSL_free(ssl_);
    if (ctx_) SSL_CTX_free(ctx_);
    if (fd_ >= 0) ::close(fd_);
  }
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;

  void set_timeout(double s) {
    timeval tv{(time_t)s, (suseconds_t)((s - (double)(time_t)s) * 1e6)};
    ::setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    ::setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  }

  // Sends a GET; returns the status and reads the response head (chunked / length / close).
  int get(const std::string& path) {
    const std::string req = "GET " + a_.prefix + path + " HTTP/1.1\r\nHost: " + a_.host +
                            "\r\nAccept: application/json\r\n" +
                            (a_.token.empty() ? "" : "Authorization: Bearer " + a_.token + "\r\n") +
                            "User-Agent: amd-node-validate\r\nConnection: keep-alive\r\n\r\n";
    for (size_t off = 0; off < req.size();) {
      const int n = ssl_ ? SSL_write(ssl_, req.data() + off, (int)(req.size() - off))
                         : (int)::send(fd_, req.data() + off, req.size() - off, MSG_NOSIGNAL);
      if (n <= 0) throw NotHandled("write to the API server failed");
      off += (size_t)n;
    }
    std::string status_line;
    if (!line(status_line) || status_line.rfind("HTTP/1.", 0) != 0) throw NotHandled("malformed API response");
    const int status = std::atoi(status_line.c_str() + status_line.find(' ') + 1);
    chunked_ = false, close_ = false, length_ = -1;
    for (std::string h; line(h) && !h.empty();) {
      std::transform(h.begin(), h.end(), h.begin(), ::tolower);
      if (h.rfind("transfer-encoding:", 0) == 0 && h.find("chunked") != std::string::npos) chunked_ = true;
      else if (h.rfind("content-length:", 0) == 0) length_ = std::atol(h.c_str() + 15);
      else if (h.rfind("connection:", 0) == 0 && h.find("close") != std::string::npos) close_ = true;
    }
    return status;
  }

  // The whole body of the last response (length-delimited, chunked, or up to the close).
  std::string body() {
    std::string out;
    if (chunked_) {
      for (std::string piece; chunk(piece);) out += piece;
    } else if (length_ >= 0) {
      if (!exact((size_t)length_, out)) throw NotHandled("short API response");
    } else {
      while (fill()) {
      }
      out.swap(buf_);
      close_ = true;
    }
    return out;
  }

  // The next chunk of a chunked body; false at its end (or when the stream breaks).
  bool chunk(std::string& out) {
    std::string size_line;
    if (!line(size_line)) return false;
    const size_t n = std::strtoul(size_line.c_str(), nullptr, 16);
    if (n == 0) {
      std::string trailer;
      while (line(trailer) && !trailer.empty()) {
      }
      return false;
    }
    out.clear();
    std::string crlf;
    return exact(n, out) && line(crlf);
  }

  bool reusable() const { return !close_; }

 private:
  void handshake() {
    ctx_ = SSL_CTX_new(TLS_client_method());
    if (a_.verify) {
      SSL_CTX_set_verify(ctx_, SSL_VERIFY_PEER, nullptr);
      bool loaded = false;
      if (!a_.ca_pem.empty()) {
        BIO* bio = BIO_new_mem_buf(a_.ca_pem.data(), (int)a_.ca_pem.size());
        while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
          loaded = X509_STORE_add_cert(SSL_CTX_get_cert_store(ctx_), x) == 1 || loaded;
          X509_free(x);
        }
        BIO_free(bio);
      } else if (!a_.ca_file.empty()) {
        loaded = SSL_CTX_load_verify_locations(ctx_, a_.ca_file.c_str(), nullptr) == 1;
      } else {
        loaded = SSL_CTX_set_default_verify_paths(ctx_) == 1;
      }
      if (!loaded) throw NotHandled("cannot load the API server CA");
    }
    ssl_ = SSL_new(ctx_);
    SSL_set_fd(ssl_, fd_);
    SSL_set_tlsext_host_name(ssl_, a_.host.c_str());
    if (a_.verify) {
      // in-cluster the API server is an IP (KUBERNETES_SERVICE_HOST): match it against the
      // certificate's IP SANs, a name against its DNS SANs
      in6_addr ip6;
      in_addr ip4;
      if (inet_pton(AF_INET, a_.host.c_str(), &ip4) == 1 || inet_pton(AF_INET6, a_.host.c_str(), &ip6) == 1)
        X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(ssl_), a_.host.c_str());
      else
        SSL_set1_host(ssl_, a_.host.c_str());
    }
    if (SSL_connect(ssl_) != 1) throw NotHandled("TLS handshake with the API server failed");
  }
  bool fill() {
    char tmp[16384];
    const int n = ssl_ ? SSL_read(ssl_, tmp, sizeof tmp) : (int)::recv(fd_, tmp, sizeof tmp, 0);
    if (n <= 0) return false;
    buf_.append(tmp, (size_t)n);
    return true;
  }
  bool line(std::string& out) {
    for (;;) {
      const auto eol = buf_.find("\r\n");
      if (eol != std::string::npos) {
        out = buf_.substr(0, eol);
        buf_.erase(0, eol + 2);
        return true;
      }
      if (!fill()) return false;
    }
  }
  bool exact(size_t n, std::string& out) {
    while (buf_.size() < n)
      if (!fill()) return false;
    out.append(buf_, 0, n);
    buf_.erase(0, n);
    return true;
  }

  const Api a_;
  int fd_ = -1;
  SSL_CTX* ctx_ = nullptr;
  SSL* ssl_ = nullptr;
  std::string buf_;
  bool chunked_ = false, close_ = false;
  long length_ = -1;
};

// --- plugin (components.validate_plugin, WITH_WORKLOAD=false) -------------------------------
// GPU resources in a Node object's capacity (amd.com/gpu; amd.com/partition-* under mixed).
long long gpu_capacity(const Value& n, bool mixed, Value& res) {
  long long devices = 0;
  const Value* st = n.find("status");
  const Value* cap = st ? st->find("capacity") : nullptr;
  if (cap && cap->is_object()) {
    for (const auto& [k, v] : cap->o) {
      if (k != "amd.com/gpu" && !(mixed && k.rfind("amd.com/partition-", 0) == 0)) continue;
      const long long c = v.is_string() ? std::atoll(v.s.c_str()) : v.integer();
      if (c > 0) {
        res[k] = Value::number(c);
        devices += c;
      }
    }
  }
  return devices;
}

// One GET of the Node, then one watch of it (fieldSelector=metadata.name) on the same kept-alive
// connection, from the resourceVersion of that GET: the device plugin's registration arrives as a
// watch event, with no polling and no connection per check. A watch the server ends (its
// timeoutSeconds, an ERROR event such as 410 Gone) is re-established from a fresh GET, at most once per
// second; a server without watches is polled every 5 s, the reference's period
// (validator/main.go:1102-1122), over the same connection.
Value validate_plugin(const Opts& o) {
  if (truthy(env("WITH_WORKLOAD", "true"))) throw NotHandled("plugin validation with a workload pod");
  if (env("VALIDATOR_WAIT_MODE") == "poll") throw NotHandled("the reference's poll mode");
  const std::string node = env("NODE_NAME");
  if (node.empty()) throw NotHandled("NODE_NAME unset");
  for (char c : node)
    if (!std::isalnum((unsigned char)c) && c != '-' && c != '.') throw NotHandled("node name " + node);
  const bool mixed = env("PARTITION_STRATEGY", env("MIG_STRATEGY", "single")) == "mixed";
  const double budget = std::atof(env("RESOURCE_TIMEOUT_SECONDS", "150").c_str());
  const Api api = api_config();
  using clock = std::chrono::steady_clock;
  const auto deadline = clock::now() + std::chrono::milliseconds((long long)(budget * 1e3));
  auto left_s = [&] { return std::chrono::duration<double>(deadline - clock::now()).count(); };
  auto found = [&](const Value& res, long long devices) {
    Value info = Value::object();
    info["resources"] = res;
    info["devices"] = Value::number(devices);
    write_barrier(o, "plugin-ready", info);
    return info;
  };
  std::unique_ptr<Conn> conn;
  bool watches = true;
  auto last_list = clock::now() - std::chrono::seconds(10);
  for (;;) {
    if (left_s() <= 0) throw ValidationError("no amd.com/gpu resources on node " + node + " after " +
                                             std::to_string((int)budget) + "s");
    if (!conn || !conn->reusable()) conn.reset(new Conn(api, 10.0));
    // the Node now (and the resourceVersion to watch from)
    const auto gap = std::chrono::duration<double>(clock::now() - last_list).count();
    const double pause = watches ? 1.0 - gap : 5.0 - gap;
    if (pause > 0) std::this_thread::sleep_for(std::chrono::milliseconds((long long)(std::min(pause, left_s()) * 1e3)));
    last_list = clock::now();
    conn->set_timeout(10.0);
    const int status = conn->get("/api/v1/nodes/" + node);
    const std::string body = conn->body();
    if (status != 200) throw NotHandled("GET node " + node + ": HTTP " + std::to_string(status));
    std::string rv;
    try {
      const Value n = minijson::parse(body);
      Value res = Value::object();
      if (const long long d = gpu_capacity(n, mixed, res)) return found(res, d);
      const Value* md = n.find("metadata");
      const Value* r = md ? md->find("resourceVersion") : nullptr;
      rv = r ? r->s : "";         // string or number text
    } catch (const NotHandled&) {
      throw;
    } catch (const std::exception& e) {
      throw NotHandled(std::string("node JSON: ") + e.what());
    }
    if (!watches) continue;
    if (!conn->reusable()) conn.reset(new Conn(api, 10.0));
    const int wait_s = std::max(1, (int)std::min(left_s(), 300.0));
    conn->set_timeout(wait_s + 10.0);
    const int ws = conn->get("/api/v1/nodes?fieldSelector=metadata.name%3D" + node + "&watch=1&timeoutSeconds=" +
                             std::to_string(wait_s) + (rv.empty() ? "" : "&resourceVersion=" + rv));
    if (ws != 200) {
      (void)conn->body();
      watches = false;      // no watches here: poll at the reference's period
      continue;
    }
    // watch events: one JSON object per line, lines split across chunks in any way
    std::string pending, piece;
    bool restart = false;
    while (!restart && conn->chunk(piece)) {
      pending += piece;
      for (size_t eol; (eol = pending.find('\n')) != std::string::npos;) {
        const std::string ev = pending.substr(0, eol);
        pending.erase(0, eol + 1);
        if (ev.find_first_not_of(" \r\t") == std::string::npos) continue;
        try {
          const Value e = minijson::parse(ev);
          const Value* type = e.find("type");
          const Value* obj = e.find("object");
          if (!type || !obj || type->str() == "ERROR") {
            restart = true;        // e.g. 410 Gone: list again
            break;
          }
          Value res = Value::object();
          if (type->str() != "DELETED")
            if (const long long d = gpu_capacity(*obj, mixed, res)) return found(res, d);
        } catch (const std::exception& e) {
          throw NotHandled(std::string("watch event JSON: ") + e.what());
        }
      }
    }
    conn.reset();   // the watch ended (server timeout, ERROR, broken stream): a new connection for the list
  }
}

// --- rccl without a fabric (components.validate_rccl, ngpu < 2) -----------------------------

Value validate_rccl(const Opts& o, int& rc) {
  std::set<std::string> phys;
  for (const auto& g : amdnode::enumerate_gpus(o.sys_root)) phys.insert(g.pci_bdf);
  const int n = (int)phys.size();
  if (n == 0 || n >= 2) {
    rc = kNotHandled;   // a fabric to prove (or no sysfs view): amd-validator plans the pod
    Value v = Value::object();
    v["physical_gpus"] = Value::number(n);
    v["handled"] = Value::boolean(false);
    return v;
  }
  Value info = Value::object();
  info["skipped"] = Value::string(std::to_string(n) + " physical GPU(s): no fabric to validate");
  info["ok"] = Value::boolean(true);
  write_barrier(o, "rccl-ready", info);
  return info;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  o.component = env("COMPONENT");
  o.with_wait = truthy(env("WITH_WAIT", "false"));
  o.out_dir = env("OUTPUT_DIR", mount_path("/run/amd/validations"));
  o.sys_root = env("AMD_SYSFS_ROOT", "/");
  o.dev_root = env("AMD_DEV_ROOT", "/");
  o.host_root = env("HOST_ROOT", mount_path("/host"));
  o.wait_timeout = std::atof(env("WAIT_TIMEOUT_SECONDS", "3600").c_str());
  o.sleep_interval = std::atof(env("SLEEP_INTERVAL_SECONDS", "5").c_str());
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--with-wait") o.with_wait = true;
    else if (a == "--output-dir") o.out_dir = next();
    else if (a == "--wait-timeout") o.wait_timeout = std::atof(next().c_str());
    else if (a == "--sys-root") o.sys_root = next();
    else if (a == "--dev-root") o.dev_root = next();
    else if (a == "--host-root") o.host_root = next();
    else if (a == "-h" || a == "--help") {
      std::printf("usage: amd-node-validate driver|toolkit|plugin|rccl [--with-wait] [--output-dir DIR] [--wait-timeout S]\n");
      return 0;
    } else if (a[0] != '-') o.component = a;
    else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  int rc = 0;
  Value info;
  try {
    if (o.component == "driver") info = validate_driver(o);
    else if (o.component == "toolkit") info = validate_toolkit(o);
    else if (o.component == "rccl") info = validate_rccl(o, rc);
    else if (o.component == "plugin") info = validate_plugin(o);
    else {
      std::fprintf(stderr, "amd-node-validate: component '%s' needs amd-validator\n", o.component.c_str());
      return kNotHandled;
    }
  } catch (const NotHandled& e) {
    std::fprintf(stderr, "amd-node-validate %s: handing over to amd-validator (%s)\n", o.component.c_str(), e.what());
    return kNotHandled;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error validating %s: %s\n", o.component.c_str(), e.what());
    return 1;
  }
  if (rc == kNotHandled) return rc;
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  Value line = Value::object();
  line["component"] = Value::string(o.component);
  line["ok"] = Value::boolean(true);
  line["seconds"] = Value::number_text(num(dt));
  line["info"] = info;
  std::printf("%s\n", minijson::dump(line).c_str());
  return 0;
}
