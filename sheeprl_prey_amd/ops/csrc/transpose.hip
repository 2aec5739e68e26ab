// Batched matrix transpose: up to 8 row-strided fp32 matrices -> contiguous transposes in ONE launch.
//
// The DreamerV3 step re-derives transposed copies of weights that changed in the last optimiser step: the
// persistent scan's W2^T / W1^T / Wg^T / Wz^T (ops/rssm.py; reference loop dreamer_v3.py:122-129 over
// agent.py:350-437) and the one-hot gather tables W[:, :S]^T of the first layers (ops/onehot.py,
// imagination at agent.py:682-739).  `.t().contiguous()` ran each as its own strided-copy launch (~7 us each,
// 13 per step).  Here: 32 x 32 tiles through LDS (row stride 33: conflict-free column reads), 256 threads
// (8 rows of 32 per pass), the tiles of every job in one grid (job found from the tile prefix sums).
#include "common.h"

namespace srl {
namespace tr {

constexpr int MAXJ = 8;
constexpr int TS = 32;

struct TJ {
  const float* src[MAXJ];
  float* dst[MAXJ];
  long lds[MAXJ];
  int rows[MAXJ], cols[MAXJ], tcols[MAXJ];  // tcols: tiles along the columns
  int tile0[MAXJ + 1];                      // prefix sums of the tile counts
  int nj;
};

__global__ void __launch_bounds__(256) transpose_kernel(TJ p) {
  __shared__ float t[TS][TS + 1];
  const int bid = blockIdx.x;
  int j = 0;
#pragma unroll
  for (int q = 1; q < MAXJ; ++q)
    if (q < p.nj && bid >= p.tile0[q]) j = q;
  const int loc = bid - p.tile0[j];
  const int tr = loc / p.tcols[j], tc = loc - tr * p.tcols[j];
  const int R = p.rows[j], Cc = p.cols[j];
  const int r0 = tr * TS, c0 = tc * TS;
  const int x = threadIdx.x & 31, y = threadIdx.x >> 5;
  const float* src = p.src[j];
#pragma unroll
  for (int k = 0; k < TS; k += 8) {
    const int r = r0 + y + k, c = c0 + x;
    if (r < R && c < Cc) t[y + k][x] = src[(long)r * p.lds[j] + c];
  }
  __syncthreads();
  float* dst = p.dst[j];
#pragma unroll
  for (int k = 0; k < TS; k += 8) {
    const int c = c0 + y + k, r = r0 + x;
    if (c < Cc && r < R) dst[(long)c * R + r] = t[x][y + k];
  }
}

}  // namespace tr
}  // namespace srl

using namespace srl;

// false: more than 8 jobs
bool launch_transpose_many(int nj, const float* const* src, const long* lds, const int* rows, const int* cols,
                           float* const* dst, hipStream_t st) {
  if (nj < 1 || nj > tr::MAXJ) return false;
  tr::TJ p{};
  p.nj = nj;
  int tiles = 0;
  for (int j = 0; j < nj; ++j) {
    p.src[j] = src[j];
    p.dst[j] = dst[j];
    p.lds[j] = lds[j];
    p.rows[j] = rows[j];
    p.cols[j] = cols[j];
    p.tcols[j] = cdiv(cols[j], tr::TS);
    p.tile0[j] = tiles;
    tiles += cdiv(rows[j], tr::TS) * p.tcols[j];
  }
  p.tile0[nj] = tiles;
  if (tiles > 0) hipLaunchKernelGGL(tr::transpose_kernel, dim3(tiles), dim3(256), 0, st, p);
  return true;
}

// One-wave delay at the head of a side-stream branch (ops/sidestream.py): holds the branch ~us microseconds of wall
// clock (s_memrealtime, 100 MHz) so that the persistent scan launched beside it claims its CUs first.
namespace srl {
__global__ void __launch_bounds__(64) side_delay_kernel(long long ticks) {
  long long t0;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < (1 << 20); ++i) {  // bounded: ends within ~10 ms whatever the clock does
    long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    if (t - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(4);
  }
}
}  // namespace srl

void launch_side_delay(float us, hipStream_t st) {
  const long long ticks = (long long)(us * 100.f);
  if (ticks > 0) hipLaunchKernelGGL(srl::side_delay_kernel, dim3(1), dim3(64), 0, st, ticks);
}
