// hiprtc-based kernel JIT (see jit.h).
#include "jit.h"

#include <hip/hiprtc.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>

#include "../common.h"

namespace tfa {
namespace jit {
namespace {

constexpr const char* kArch = "gfx950";

std::mutex g_mu;
std::map<std::string, std::vector<char>> g_code;               // key -> code object
std::map<std::pair<std::string, int>, hipModule_t> g_modules;  // (key, device) -> module
std::map<std::tuple<std::string, int, std::string>, hipFunction_t> g_funcs;
Stats g_stats;

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

std::vector<std::string> options() {
  // no fused multiply-add in the generated elementwise kernels: they round
  // after every op like the CPU executor (and the image pre-stage kernel),
  // so a fused chain gives the host oracle's bits; they are memory-bound
  return {std::string("--offload-arch=") + kArch, "-O3", "-std=c++17", "-ffp-contract=off"};
}

std::string key_of(const std::string& src) {
  std::string all = src;
  for (auto& o : options()) all += "\n//opt " + o;
  char buf[40];
  std::snprintf(buf, sizeof(buf), "%016llx%08x", static_cast<unsigned long long>(fnv1a(all)),
                static_cast<unsigned>(fnv1a(all, 0x84222325cbf29ce4ull) & 0xffffffffu));
  return buf;
}

bool make_dirs(const std::string& path) {
  std::string cur;
  std::stringstream ss(path);
  std::string part;
  if (!path.empty() && path[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
  }
  return true;
}

std::string cache_dir() {
  static const std::string dir = [] {
    std::vector<std::string> cands;
    if (const char* e = std::getenv("TFA_JIT_CACHE_DIR")) cands.push_back(e);
    if (const char* x = std::getenv("XDG_CACHE_HOME")) cands.push_back(std::string(x) + "/tensorframes_amd/jit");
    if (const char* h = std::getenv("HOME")) cands.push_back(std::string(h) + "/.cache/tensorframes_amd/jit");
    cands.push_back("/tmp/tensorframes_amd_jit_" + std::to_string(getuid()));
    for (auto& c : cands)
      if (make_dirs(c) && access(c.c_str(), W_OK) == 0) return c;
    return std::string();
  }();
  return dir;
}

bool disk_cache_enabled() {
  const char* e = std::getenv("TFA_JIT_DISK_CACHE");
  return !(e && e[0] == '0');
}

bool read_file(const std::string& path, std::vector<char>* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  out->assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return !out->empty();
}

void write_file_atomic(const std::string& path, const std::vector<char>& data) {
  std::string tmp = path + ".tmp" + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::binary);
    if (!f) return;
    f.write(data.data(), static_cast<std::streamsize>(data.size()));
    if (!f) return;
  }
  std::rename(tmp.c_str(), path.c_str());
}

std::vector<char> compile(const std::string& src) {
  auto t0 = std::chrono::steady_clock::now();
  hiprtcProgram prog;
  TFA_CHECK(hiprtcCreateProgram(&prog, src.c_str(), "tfa_fused.hip", 0, nullptr, nullptr) == HIPRTC_SUCCESS,
            "hiprtcCreateProgram failed");
  auto opts = options();
  std::vector<const char*> copts;
  for (auto& o : opts) copts.push_back(o.c_str());
  hiprtcResult r = hiprtcCompileProgram(prog, static_cast<int>(copts.size()), copts.data());
  if (r != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    TFA_CHECK(false, "JIT compile of a fused kernel failed (", hiprtcGetErrorString(r), "):\n", log,
              "\n--- source ---\n", src);
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  std::vector<char> code(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  g_stats.compiled++;
  g_stats.compile_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return code;
}

const std::vector<char>& code_for(const std::string& src, const std::string& key) {
  auto it = g_code.find(key);
  if (it != g_code.end()) {
    g_stats.memory_hits++;
    return it->second;
  }
  std::vector<char> code;
  std::string path;
  if (disk_cache_enabled() && !cache_dir().empty()) {
    path = cache_dir() + "/" + key + ".co";
    if (read_file(path, &code)) g_stats.disk_hits++;
  }
  if (code.empty()) {
    code = compile(src);
    if (!path.empty()) write_file_atomic(path, code);
  }
  return g_code.emplace(key, std::move(code)).first->second;
}

}  // namespace

Kernel get(const std::string& source, const std::string& entry) {
  std::lock_guard<std::mutex> lk(g_mu);
  const std::string key = key_of(source);
  int dev = 0;
  TFA_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice failed");
  auto fk = std::make_tuple(key, dev, entry);
  auto fit = g_funcs.find(fk);
  if (fit != g_funcs.end()) return Kernel{fit->second, entry};
  hipModule_t mod = nullptr;
  auto mit = g_modules.find({key, dev});
  if (mit != g_modules.end()) {
    mod = mit->second;
  } else {
    const std::vector<char>& code = code_for(source, key);
    hipError_t e = hipModuleLoadData(&mod, code.data());
    TFA_CHECK(e == hipSuccess, "hipModuleLoadData of a fused kernel failed: ", hipGetErrorString(e));
    g_modules[{key, dev}] = mod;
  }
  hipFunction_t fn = nullptr;
  hipError_t e = hipModuleGetFunction(&fn, mod, entry.c_str());
  TFA_CHECK(e == hipSuccess, "hipModuleGetFunction(", entry, ") failed: ", hipGetErrorString(e));
  g_funcs[fk] = fn;
  return Kernel{fn, entry};
}

size_t compile_only(const std::string& source) {
  std::lock_guard<std::mutex> lk(g_mu);
  return code_for(source, key_of(source)).size();
}

void launch(const Kernel& k, unsigned grid, unsigned block, const void* args, size_t args_size,
            hipStream_t stream) {
  TFA_CHECK(k.fn != nullptr, "launch of an unloaded JIT kernel");
  TFA_CHECK(grid >= 1 && block >= 1 && block <= 1024, "JIT launch: bad geometry ", grid, "x", block);
  size_t sz = args_size;
  void* config[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, const_cast<void*>(args), HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                    HIP_LAUNCH_PARAM_END};
  hipError_t e = hipModuleLaunchKernel(k.fn, grid, 1, 1, block, 1, 1, 0, stream, nullptr, config);
  TFA_CHECK(e == hipSuccess, "hipModuleLaunchKernel(", k.name, ") failed: ", hipGetErrorString(e));
}

Stats stats() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_stats;
}

}  // namespace jit
}  // namespace tfa
