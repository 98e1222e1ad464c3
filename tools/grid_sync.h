// Grid-wide barrier for persistent kernels on MI355X (8 XCDs x 32 CUs, one
// private L2 per XCD): XCD-hierarchical arrival, relaxed polling, one
// agent-scope acquire after the exit.
//
//   arrive   every storing wave drains its stores (s_waitcnt vmcnt(0)), the
//            workgroup barrier, then ONE lane: agent-scope release fence
//            (writes back this XCD's dirty L2 lines: cheap when the bulk
//            payload was stored write-through, sc1) and one agent-scope
//            atomic add on its group's counter.  Groups are blockIdx % 8
//            (a label that matches the dispatcher's round-robin XCD
//            placement: speed only, never correctness), so 32 arrivals
//            share a counter instead of 256.
//   release  the last arriver of a group adds to the top counter; the last
//            group's arriver bumps the top generation word; each group's
//            last arriver polls that word and then releases its group's
//            generation word, which the group's other workgroups poll.
//   wait     relaxed agent-scope loads with s_sleep between polls (an
//            acquire per poll pays an L1 invalidate each time), then ONE
//            agent-scope acquire fence (buffer_inv sc1) and a workgroup
//            barrier: every wave's later plain loads see the other
//            workgroups' stores.
//
// Counters are monotonic within a launch (epoch e = 1, 2, ...: the barrier's
// ordinal), zeroed by the host before every launch.  Every spin is bounded:
// a workgroup that polls past the limit sets the timeout word and the
// barrier returns false on every thread of that workgroup; the caller must
// then leave the kernel (so the grid always drains, and the host raises).
// Residency: the caller launches at most as many workgroups as are
// co-resident (CUs x blocks per CU of its LDS / VGPR budget).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace twtml {

constexpr int kSyncGroups = 8;
constexpr int kSyncLine = 32;   // u32 words per 128-B line: one counter per line
// word layout: [g * line] group counters, [8 line] top counter,
// [(9 + g) line] group generations, [17 line] top generation, [18 line] timeout
constexpr int kSyncWords = 19 * kSyncLine;
constexpr uint32_t kSyncSpinLimit = 1u << 21;   // polls (s_sleep 2 each): ~0.5 s

using gu32 = __attribute__((address_space(1))) uint32_t;

__device__ __forceinline__ gu32* sync_word(uint32_t* words, int idx) {
  return (gu32*)(words + idx);   // generic -> global address space
}

// One lane polls `w` until it reaches `target` (relaxed, s_sleep between
// polls); false after kSyncSpinLimit polls (timeout word set).
__device__ __forceinline__ bool sync_poll(uint32_t* words, int idx, uint32_t target) {
  gu32* w = sync_word(words, idx);
  for (uint32_t spins = 0;; ++spins) {
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    if (spins >= kSyncSpinLimit) {
      __hip_atomic_store(sync_word(words, 18 * kSyncLine), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Barrier `epoch` (1-based ordinal within the launch) over `nblocks`
// workgroups.  Every thread of every workgroup calls it; returns false on
// every thread of a workgroup that timed out.
__device__ __forceinline__ bool grid_sync(uint32_t* words, uint32_t epoch, uint32_t nblocks) {
  __shared__ uint32_t ok_s;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores have left the CU
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t g = blockIdx.x % kSyncGroups;
    const uint32_t gsize = (nblocks + kSyncGroups - 1 - g) / kSyncGroups;
    const uint32_t ngroups = nblocks < uint32_t(kSyncGroups) ? nblocks : uint32_t(kSyncGroups);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool ok = true;
    const uint32_t prev = __hip_atomic_fetch_add(sync_word(words, int(g) * kSyncLine), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == epoch * gsize - 1) {   // last of its group: arrive at the top
      const uint32_t top = __hip_atomic_fetch_add(sync_word(words, 8 * kSyncLine), 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      if (top == epoch * ngroups - 1)
        __hip_atomic_store(sync_word(words, 17 * kSyncLine), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        ok = sync_poll(words, 17 * kSyncLine, epoch);
      __hip_atomic_store(sync_word(words, (9 + int(g)) * kSyncLine), epoch, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);   // release the group (also on timeout: it drains)
    } else {
      ok = sync_poll(words, (9 + int(g)) * kSyncLine, epoch);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ok_s = ok ? 1u : 0u;
  }
  __syncthreads();
  return ok_s != 0u;
}

// Host: bytes of the barrier's word block (zero it before every launch).
constexpr size_t kSyncBytes = size_t(kSyncWords) * sizeof(uint32_t);

}  // namespace twtml
