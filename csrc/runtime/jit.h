// Runtime kernel compilation for gfx950 (hiprtc) with an in-memory and an
// on-disk code-object cache.
//
// The planner generates HIP source for fused regions of the graph (elementwise
// chains, reduction prologues; runtime/fusion.*). Source text is compiled once
// per process (≈20-40 ms after hiprtc's first ≈2 s load), code objects are kept
// on disk under TFA_JIT_CACHE_DIR (default ~/.cache/tensorframes_amd/jit, else
// /tmp), keyed by a hash of source + options, and loaded per device with
// hipModuleLoadData. The reference has no counterpart: TF 1.1 CPU ran every
// op separately (SURVEY.md §2.3 "Fused ops").
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace tfa {
namespace jit {

struct Kernel {
  hipFunction_t fn = nullptr;
  std::string name;
};

// Compile (or fetch from cache) `source` and return the `entry` kernel for
// the current device. Throws GraphError with the compiler log on failure.
Kernel get(const std::string& source, const std::string& entry);

// Compile only (no device needed): returns the code object size, throws on
// error. Used by CPU tests of the code generator.
size_t compile_only(const std::string& source);

// Launch with the kernel arguments packed in one POD struct (passed by value
// as the kernel's single parameter).
void launch(const Kernel& k, unsigned grid, unsigned block, const void* args, size_t args_size,
            hipStream_t stream);

struct Stats {
  int64_t compiled = 0, disk_hits = 0, memory_hits = 0;
  double compile_ms = 0;
};
Stats stats();

}  // namespace jit
}  // namespace tfa
