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

}  // namespace gather
}  // namespace srl

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
