// Cross-workgroup reductions and non-finite guards shared by the training
// kernels (dttrain.hip, dtupd.hip): Chan's merge, write-through partials, the
// last-arrival hand-off with its agent-scope acquire, guard reports
// (include/dttrain.h DT_GUARD_*).
#ifndef AIDO1_AMD_DTSYNC_H
#define AIDO1_AMD_DTSYNC_H

#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

// Chan et al.: merge (nb, mb, m2b) into (n, mean, m2).  Merges run in long
// dependent chains (a workgroup's waves, the partials of a launch), so the
// weight nb / tot takes the hardware reciprocal (1 ulp) instead of an IEEE
// division (a dozen dependent instructions); merging into an empty side
// copies exactly.
__device__ __forceinline__ void chan(float& n, float& mean, float& m2, float nb, float mb,
                                     float m2b) {
  if (nb <= 0.0f) return;
  if (n <= 0.0f) {
    n = nb;
    mean = mb;
    m2 = m2b;
    return;
  }
  const float tot = n + nb;
  const float d = mb - mean;
  const float f = nb * __builtin_amdgcn_rcpf(tot);
  mean += d * f;
  m2 += m2b + d * d * n * f;
  n = tot;
}

// Partials cross workgroups (and XCDs, whose L2s are not coherent): they are
// written through to memory (agent-scope relaxed atomic stores: `sc1`, the
// line leaves the XCD's L2), so no release fence has to write back the L2
// full of this launch's activations, and read back by the last arriver
// behind an agent-scope acquire (`acquire_partials`): MI355X_MICROARCH.md's
// consumer form for any placement of the workgroups (the `sc1`-loads-only
// form is measured for one workgroup a CU, and two of these 1024-thread
// workgroups fit a CU beside other streams' kernels).
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// true for the workgroup that arrives last at `counter` (which it resets);
// every workgroup's write-through partials have landed before it arrives
__device__ bool last_arrival(unsigned int* counter) {
  __shared__ bool last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int old =
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1;
    if (last) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return last;
}

// the last arriver, before its first load of another workgroup's partials:
// one wave invalidates the CU's L1 (agent acquire) and waits for it, the
// barrier holds every wave until then
__device__ __forceinline__ void acquire_partials() {
  if (threadIdx.x < 64) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

__device__ __forceinline__ bool finitef(float x) { return fabsf(x) <= 3.402823466e38f; }

// one lane of each wave that saw a non-finite value (`bad`) reports it:
// guard[0] |= 1 << bit, guard[1] += 1, guard[3 + bit] = min(., tick)
__device__ __forceinline__ void guard_raise(int32_t* guard, int bit, bool bad) {
  if (!guard || bit < 0) return;
  const unsigned long long b = __ballot(bad);
  if (b == 0) return;
  if ((int)(threadIdx.x & 63) == __ffsll((long long)b) - 1) {
    atomicOr(&guard[0], 1 << bit);
    atomicAdd(&guard[1], 1);
    atomicMin(&guard[3 + bit], guard[2]);
  }
}

}  // namespace

#endif  // AIDO1_AMD_DTSYNC_H
