// mfa_launch.h — the one way every kernel of the library is launched.
//
// Two jobs:
//   * the dynamic-LDS attribute (hipFuncAttributeMaxDynamicSharedMemorySize) is set once per
//     (kernel, device) under a mutex, so host threads driving different devices in one
//     process neither race nor skip a device or an instantiation;
//   * plan capture: while a thread has a capture record installed (mfa_multihead_plan,
//     mfa_attention_kernel_create in mfa_api.cpp), a launch records the kernel instantiation
//     (its exported symbol, the name rocprofv3 shows), workgroup size, LDS bytes and grid
//     instead of launching.  The plan API therefore runs
//     the real dispatcher and reports exactly what a call with the same arguments launches
//     (the reference's AttentionKernel is the thing it dispatches, AttentionKernel.swift:23-32).
#pragma once
#include <hip/hip_runtime.h>

#include <cxxabi.h>
#include <dlfcn.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <utility>


namespace mfa {

// Development A/B switches (MFA_FWD_SHARE, MFA_KV_REGS, MFA_GEMM3, ...) change which kernel a
// call launches.  They are read only in a process started with MFA_DEV=1 (the test suite and
// the A/B tools set it; read once, at the first dispatch), so a production caller's
// environment can never change the plan, and the dispatch path calls no getenv otherwise.
inline const char* dev_env(const char* name) {
  static const bool dev = [] {
    const char* e = std::getenv("MFA_DEV");
    return e != nullptr && e[0] == '1' && e[1] == 0;
  }();
  return dev ? std::getenv(name) : nullptr;
}

struct LaunchRec {
  char name[96];
  uint32_t threads;
  uint32_t lds_bytes;
  uint64_t workgroups;
};

struct PlanCapture {
  static constexpr int kMax = 4;
  LaunchRec rec[kMax];
  int count = 0;   // recorded (at most kMax)
  int total = 0;   // issued
};

// Installed by the plan API for the duration of one dispatch on this thread (mfa_api.cpp).
// Inline with vague linkage: one slot per thread across every translation unit of the library.
inline PlanCapture*& plan_capture() {
  static thread_local PlanCapture* cap = nullptr;
  return cap;
}

// The attribute state is keyed by (kernel handle, device): every instantiation gets its own
// hipFuncSetAttribute on every device, whatever its signature.  The value set is the largest
// LDS size a launch of that kernel has asked for so far on that device.
struct LdsAttrTable {
  std::mutex mu;
  std::map<std::pair<const void*, int>, std::pair<size_t, hipError_t>> set;
};
inline LdsAttrTable& lds_attr_table() {
  static LdsAttrTable t;
  return t;
}

inline hipError_t set_lds_attr_per_device(const void* kern, size_t bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  LdsAttrTable& t = lds_attr_table();
  std::lock_guard<std::mutex> lock(t.mu);
  // Only successful sets are remembered (the largest size set so far): a failed request is
  // retried by the next launch instead of failing every later one of that kernel.
  auto it = t.set.find({kern, dev});
  if (it != t.set.end() && it->second.first >= bytes) return hipSuccess;
  e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) t.set[{kern, dev}] = {bytes, e};
  return e;
}

// Number of (kernel, device) pairs whose LDS attribute has been set (tests).
inline size_t lds_attr_entries() {
  LdsAttrTable& t = lds_attr_table();
  std::lock_guard<std::mutex> lock(t.mu);
  return t.set.size();
}

// Launch log: the handles and shapes of the launches this thread issued since the log was
// last read (mfa_last_launches), kept so a caller can check a plan against what ran.  Only
// pointers and sizes are stored on the launch path; names are resolved when read.
struct LaunchLog {
  static constexpr int kMax = 8;
  const void* handle[kMax];
  uint32_t threads[kMax], lds[kMax];
  uint64_t workgroups[kMax];
  uint64_t total = 0;
};
inline LaunchLog& launch_log() {
  static thread_local LaunchLog log;
  return log;
}

// The kernel's name as rocprofv3 reports it, shortened the way tools/pmc_traffic.py keys its
// records: the handle's exported symbol, demangled, without "void ", "mfa::" qualifiers and
// the parameter list ("mfa_fwd2_pair_kernel<F16, 128, 64, 4>").  Host-only, no GPU needed.
inline void kernel_symbol_name(const void* handle, char* out, size_t n) {
  Dl_info info;
  if (!dladdr(handle, &info) || !info.dli_sname || info.dli_saddr != handle) {
    snprintf(out, n, "?");
    return;
  }
  int status = 0;
  char* dem = abi::__cxa_demangle(info.dli_sname, nullptr, nullptr, &status);
  std::string s = (status == 0 && dem) ? dem : info.dli_sname;
  free(dem);
  if (s.rfind("void ", 0) == 0) s.erase(0, 5);
  for (size_t p; (p = s.find("mfa::")) != std::string::npos;) s.erase(p, 5);
  if (!s.empty() && s.back() == ')') {
    int depth = 0;
    for (size_t i = s.size(); i-- > 0;) {
      depth += s[i] == ')' ? 1 : s[i] == '(' ? -1 : 0;
      if (depth == 0) {
        s.erase(i);
        break;
      }
    }
  }
  snprintf(out, n, "%s", s.c_str());
}

// Launches kern<<<grid, block, lds, stream>>>(args...), or records it while a plan is captured.
template <class K, class... Args>
inline hipError_t launch(K kern, dim3 grid, dim3 block, size_t lds, hipStream_t stream,
                         const Args&... args) {
  if (PlanCapture* cap = plan_capture()) {
    ++cap->total;
    if (cap->count < PlanCapture::kMax) {
      LaunchRec& r = cap->rec[cap->count++];
      kernel_symbol_name((const void*)kern, r.name, sizeof(r.name));
      r.threads = block.x * block.y * block.z;
      r.lds_bytes = (uint32_t)lds;
      r.workgroups = (uint64_t)grid.x * grid.y * grid.z;
    }
    return hipSuccess;
  }
  if (lds > 0) {
    hipError_t e = set_lds_attr_per_device((const void*)kern, lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, grid, block, lds, stream, args...);
  LaunchLog& log = launch_log();
  const int i = (int)(log.total++ % LaunchLog::kMax);
  log.handle[i] = (const void*)kern;
  log.threads[i] = block.x * block.y * block.z;
  log.lds[i] = (uint32_t)lds;
  log.workgroups[i] = (uint64_t)grid.x * grid.y * grid.z;
  return hipGetLastError();
}

}  // namespace mfa
