// Hand-off latency between workgroups on the SAME XCD vs on DIFFERENT XCDs (verdict r4 "next round" #1, step 1-2:
// measure before re-partitioning the persistent RSSM scan around XCD locality).
//
// The persistent scan's protocol (rssm_persist.hip: write-through sc1 payload stores, s_waitcnt vmcnt(0), barrier,
// one lane adds to a sharded arrival counter; the consumer polls the shards with sc1 loads, then reads the payload
// with sc1 loads) is run as a chain of NP producers -> NC consumers -> NP producers ... for R rounds.  Every
// workgroup reads its XCD from HW_REG_XCC_ID and takes a ticket from its XCD's counter; the roles are picked by
// (XCD, ticket), so the same binary measures:
//   same : producers and consumers on XCD 0
//   cross: producers on XCD 0, consumers on XCD 1
//   spread: producers and consumers dealt over all 8 XCDs (the scan's current placement)
// Payload per producer per round: 16 rows x 16 floats (one scan tile, 1 KB).  Workgroups without a role exit at once.
// Every wait is bounded; a timeout sets the error word and every waiter leaves.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o xcd_handoff xcd_handoff.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32;

constexpr int NTH = 256;
constexpr int MAXP = 32;        // producers / consumers per role
constexpr int NSH = 8, SHW = 32;  // counter shards (128-B apart)
constexpr u32 SPIN = 1u << 22;

__device__ __forceinline__ long long rtc() {
  long long c;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c)::"memory");
  return c;
}
__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct Args {
  u32* tickets;   // [8] per-XCD tickets
  u32* ctr;       // [2 roles][NSH * SHW] arrival counters
  u32* err;
  float* payload; // [2 roles][MAXP][256]
  long long* out; // [2]: total ticks measured by producer 0 / consumer 0
  int mode;       // 0 same, 1 cross, 2 spread
  int np, nc, rounds;
};

// wave 0 polls every shard until it holds `need` arrivals in total (sum over shards)
__device__ bool wait_all(const Args& a, u32* c, u32 need, int* flag) {
  if (threadIdx.x < 64) {
    int bad = 0;
    for (u32 s = 0;; ++s) {
      u32 v = threadIdx.x < NSH ? __hip_atomic_load(c + threadIdx.x * SHW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
      const u32 e = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (e) { bad = 1; break; }
      if (v >= need) break;
      if (s >= SPIN) { bad = 2; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (threadIdx.x == 0) {
      if (bad == 2) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = bad;
    }
  }
  __syncthreads();
  const bool ok = *flag == 0;
  __syncthreads();
  return ok;
}

__global__ void __launch_bounds__(NTH) handoff_kernel(Args a) {
  __shared__ int flag;
  __shared__ int role_s, idx_s;
  __shared__ float stage[MAXP * 16];
  if (threadIdx.x == 0) {
    const int x = xcc_id();
    const u32 t = __hip_atomic_fetch_add(a.tickets + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int role = -1, idx = -1;
    if (a.mode == 0) {  // same XCD: tickets 0..np-1 produce, np..np+nc-1 consume, all on XCD 0
      if (x == 0 && (int)t < a.np) role = 0, idx = t;
      else if (x == 0 && (int)t < a.np + a.nc) role = 1, idx = t - a.np;
    } else if (a.mode == 1) {  // producers on XCD 0, consumers on XCD 1
      if (x == 0 && (int)t < a.np) role = 0, idx = t;
      else if (x == 1 && (int)t < a.nc) role = 1, idx = t;
    } else {  // spread: producer i on XCD i % 8, consumer j on XCD j % 8 (ticket = slot within the XCD)
      const int per_p = (a.np + 7) / 8, per_c = (a.nc + 7) / 8;
      if ((int)t < per_p && (int)t * 8 + x < a.np) role = 0, idx = t * 8 + x;
      else if ((int)t >= per_p && (int)t < per_p + per_c && ((int)t - per_p) * 8 + x < a.nc) role = 1, idx = ((int)t - per_p) * 8 + x;
    }
    role_s = role;
    idx_s = idx;
  }
  __syncthreads();
  const int role = role_s, idx = idx_s;
  if (role < 0) return;
  u32* cp = a.ctr;            // producers arrive here
  u32* cc = a.ctr + NSH * SHW;  // consumers arrive here
  const int nmine = role == 0 ? a.np : a.nc, nother = role == 0 ? a.nc : a.np;
  float* mine = a.payload + (size_t)role * MAXP * 256 + (size_t)idx * 256;
  const float* other = a.payload + (size_t)(1 - role) * MAXP * 256;
  long long t0 = 0;
  for (int r = 0; r < a.rounds; ++r) {
    if (r == 1) t0 = rtc();  // round 0 absorbs the launch skew
    if (role == 1 || r > 0) {
      // wait for every workgroup of the other role's round r (consumers) / r - 1 (producers)
      const u32 need = (u32)nother * (u32)(role == 1 ? r + 1 : r);
      if (!wait_all(a, role == 1 ? cp : cc, need, &flag)) return;
      // read every handed-off tile (sc1 loads), one float per thread per tile, summed into LDS
      float s = 0.f;
      for (int q = 0; q < nother; ++q) s += __hip_atomic_load(const_cast<float*>(other) + q * 256 + threadIdx.x, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
      stage[threadIdx.x & (MAXP * 16 - 1)] = s;
      __syncthreads();
    }
    // publish this workgroup's tile (write-through), drain, join, one lane arrives on its shard
    __hip_atomic_store(mine + threadIdx.x, (float)(r + idx) + stage[threadIdx.x & (MAXP * 16 - 1)] * 0.f, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    drain();
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add((role == 0 ? cp : cc) + (idx % NSH) * SHW, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (idx == 0 && threadIdx.x == 0) a.out[role] = rtc() - t0;
  (void)nmine;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
  u32 *tickets, *ctr, *err;
  float* payload;
  long long* out;
  hipMalloc(&tickets, 8 * sizeof(u32));
  hipMalloc(&ctr, 2 * NSH * SHW * sizeof(u32));
  hipMalloc(&err, sizeof(u32));
  hipMalloc(&payload, 2 * MAXP * 256 * sizeof(float));
  hipMalloc(&out, 2 * sizeof(long long));
  hipFuncSetAttribute(reinterpret_cast<const void*>(handoff_kernel), hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  const char* names[3] = {"same XCD", "cross XCD (P on 0, C on 1)", "spread over 8 XCDs"};
  const int cfg[][2] = {{1, 1}, {4, 4}, {8, 8}, {16, 16}, {8, 24}};
  printf("rounds %d; one round = producers publish 1 KB tiles -> consumers wait all + read all -> consumers publish -> producers wait all + read all\n", rounds);
  printf("%-30s %4s %4s %12s %12s\n", "placement", "np", "nc", "us/round", "us/hand-off");
  for (int mode = 0; mode < 3; ++mode) {
    for (auto& c : cfg) {
      const int np = c[0], nc = c[1];
      if (mode < 2 && np + nc > 32 && mode == 0) continue;  // one XCD has 32 CUs
      hipMemset(tickets, 0, 8 * sizeof(u32));
      hipMemset(ctr, 0, 2 * NSH * SHW * sizeof(u32));
      hipMemset(err, 0, sizeof(u32));
      hipMemset(out, 0, 2 * sizeof(long long));
      Args a{tickets, ctr, err, payload, out, mode, np, nc, rounds};
      // 256 workgroups (one per CU: 40 KB static + dynamic LDS keeps it one per CU), most exit at once
      hipLaunchKernelGGL(handoff_kernel, dim3(256), dim3(NTH), 96 * 1024, 0, a);
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
      u32 e = 0;
      long long o[2];
      hipMemcpy(&e, err, sizeof(u32), hipMemcpyDeviceToHost);
      hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
      const double us = o[0] / 100.0 / (rounds - 1);  // s_memrealtime: 100 MHz
      printf("%-30s %4d %4d %12.3f %12.3f%s\n", names[mode], np, nc, us, us / 2, e ? "  (TIMEOUT)" : "");
    }
  }
  return 0;
}
