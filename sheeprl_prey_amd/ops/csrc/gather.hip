// Replay-buffer sequence gather (reference data/buffers.py SequentialReplayBuffer._get_samples): every
// key of a sample is a row gather  dst[n] = src[row[n], env[n]]  from the HBM-resident store
// [capacity, n_envs, feat...].  One launch moves all keys (up to 16): workgroup (n, key) copies one
// row with 16-byte vectors when the row size allows it, 4-byte words or bytes otherwise.
#include "common.h"

#include <algorithm>

namespace srl {
namespace gather {

constexpr int MAXK = 16;

struct GP {
  const unsigned char* src[MAXK];
  unsigned char* dst[MAXK];
  long row_bytes[MAXK];
  int nk, n_envs, N;
  long cap;  // rows of the store: indices outside [0, cap) x [0, n_envs) are never dereferenced
  const long* row;  // [N]
  const long* env;  // [N]
  int* err;         // optional: set to 1 when an index was out of range (read off the hot path)
};

__global__ __launch_bounds__(256) void gather_rows_kernel(GP p) {
  const int n = blockIdx.x, k = blockIdx.y;
  if (k >= p.nk || n >= p.N) return;
  const long rb = p.row_bytes[k];
  const long ri = p.row[n], ei = p.env[n];
  unsigned char* d = p.dst[k] + (long)n * rb;
  if (ri < 0 || ri >= p.cap || ei < 0 || ei >= p.n_envs) {
    // an out-of-range index is a caller bug: the row comes back zero-filled (never stale memory) and the
    // error word is raised for the host check (SequentialReplayBuffer.check_gather_error)
    for (long i = threadIdx.x; i < rb; i += 256) d[i] = 0;
    if (threadIdx.x == 0 && p.err != nullptr) atomicOr(p.err, 1);
    return;
  }
  const unsigned char* s = p.src[k] + (ri * p.n_envs + ei) * rb;
  if ((rb & 15) == 0 && (reinterpret_cast<uintptr_t>(s) & 15) == 0 && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
    const long n16 = rb >> 4;
    for (long i = threadIdx.x; i < n16; i += 256) reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
  } else if ((rb & 3) == 0 && (reinterpret_cast<uintptr_t>(s) & 3) == 0 && (reinterpret_cast<uintptr_t>(d) & 3) == 0) {
    const long n4 = rb >> 2;
    for (long i = threadIdx.x; i < n4; i += 256) reinterpret_cast<unsigned*>(d)[i] = reinterpret_cast<const unsigned*>(s)[i];
  } else {
    for (long i = threadIdx.x; i < rb; i += 256) d[i] = s[i];
  }
}

// Fused sequence sample (SequentialReplayBuffer.sample + the copy into a graph's static inputs): the start
// row of sample b is drawn on the device - uniform over the valid starts [0, n1) U [start2, start2 + n2) - and
// its env uniform over [0, n_envs), from a counter-based hash (splitmix64 of seed, call counter, b), so the
// host issues ONE launch per gradient step instead of ~15 small ATen ops (index draw, arange, modulo, gather,
// copy-in) - the host, not the GPU, bounds that part of the env-interaction step.  Output row (t, b) lands at
// dst[k] + (t * B + b) * row_bytes: the [T, B] layout the train step reads.
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ long uniform_below(unsigned long long h, long n) {
  // 53 random bits -> [0, n)
  const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  long v = (long)(u * (double)n);
  return v < n ? v : n - 1;
}

struct SP {
  const unsigned char* src[MAXK];
  unsigned char* dst[MAXK];
  long row_bytes[MAXK];
  int nk, n_envs, B, L;
  long cap, n1, start2, n2;
  unsigned long long seed, counter;
};

__global__ __launch_bounds__(256) void seq_sample_kernel(SP p) {
  const int n = blockIdx.x, k = blockIdx.y;
  if (k >= p.nk || n >= p.B * p.L) return;
  const int t = n / p.B, b = n - t * p.B;
  const unsigned long long h0 = splitmix64(p.seed ^ splitmix64(p.counter * 0x100000001B3ull + (unsigned long long)b));
  const long kk = uniform_below(h0, p.n1 + p.n2);
  const long start = kk < p.n1 ? kk : p.start2 + (kk - p.n1);
  const long ei = p.n_envs > 1 ? uniform_below(splitmix64(h0), p.n_envs) : 0;
  long ri = (start + t) % p.cap;
  const long rb = p.row_bytes[k];
  const unsigned char* s = p.src[k] + (ri * p.n_envs + ei) * rb;
  unsigned char* d = p.dst[k] + (long)n * rb;
  if ((rb & 15) == 0 && (reinterpret_cast<uintptr_t>(s) & 15) == 0 && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
    const long n16 = rb >> 4;
    for (long i = threadIdx.x; i < n16; i += 256) reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
  } else if ((rb & 3) == 0 && (reinterpret_cast<uintptr_t>(s) & 3) == 0 && (reinterpret_cast<uintptr_t>(d) & 3) == 0) {
    const long n4 = rb >> 2;
    for (long i = threadIdx.x; i < n4; i += 256) reinterpret_cast<unsigned*>(d)[i] = reinterpret_cast<const unsigned*>(s)[i];
  } else {
    for (long i = threadIdx.x; i < rb; i += 256) d[i] = s[i];
  }
}

}  // namespace gather
}  // namespace srl

bool launch_seq_sample(const void* const* src, void* const* dst, const long* row_bytes, int nk, int n_envs, long cap, int B,
                       int L, long n1, long start2, long n2, unsigned long long seed, unsigned long long counter,
                       hipStream_t st) {
  if (nk < 1 || nk > srl::gather::MAXK || B < 1 || L < 1 || n1 + n2 < 1 || n1 < 0 || n2 < 0 || start2 < 0 ||
      start2 + n2 > cap || n1 > cap)
    return false;
  srl::gather::SP p{};
  p.nk = nk;
  for (int k = 0; k < nk; ++k) {
    p.src[k] = static_cast<const unsigned char*>(src[k]);
    p.dst[k] = static_cast<unsigned char*>(dst[k]);
    p.row_bytes[k] = row_bytes[k];
  }
  p.n_envs = n_envs;
  p.cap = cap;
  p.B = B;
  p.L = L;
  p.n1 = n1;
  p.start2 = start2;
  p.n2 = n2;
  p.seed = seed;
  p.counter = counter;
  hipLaunchKernelGGL(srl::gather::seq_sample_kernel, dim3(B * L, nk), dim3(256), 0, st, p);
  return true;
}

void launch_gather_rows(const void* const* src, void* const* dst, const long* row_bytes, int nk, int n_envs, long cap, int N,
                        const long* row, const long* env, int* err, hipStream_t st) {
  srl::gather::GP p{};
  p.err = err;
  p.cap = cap;
  p.nk = std::min(nk, srl::gather::MAXK);
  for (int k = 0; k < p.nk; ++k) {
    p.src[k] = static_cast<const unsigned char*>(src[k]);
    p.dst[k] = static_cast<unsigned char*>(dst[k]);
    p.row_bytes[k] = row_bytes[k];
  }
  p.n_envs = n_envs;
  p.N = N;
  p.row = row;
  p.env = env;
  hipLaunchKernelGGL(srl::gather::gather_rows_kernel, dim3(N, p.nk), dim3(256), 0, st, p);
}
