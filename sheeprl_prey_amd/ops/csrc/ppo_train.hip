// One-launch PPO update for MLP agents (reference: ppo/ppo.py:32-104 train loop, ppo/loss.py:6-72,
// discrete policy head ppo/agent.py:134-178; optimiser torch.optim.Adam semantics as FlatAdam).
//
// A CartPole-sized PPO update is update_epochs x (n / batch) = 20 minibatch steps of ~25k-parameter
// MLPs: as kernels + autograd that is ~140 launches per step, each ~4 us of launch/latency for a few
// thousand FLOPs.  Here ONE workgroup (8 waves) runs the whole update:
//   * the weights stay in LDS for the entire launch, transposed and bias-augmented (W^T with b as
//     row din, row stride padded to dout+4 floats so column reads over k are bank-conflict-free);
//   * each minibatch is processed in chunks of 16 rows: forward through encoder / actor / head /
//     critic (activations in LDS with a constant-1 "bias input" column), the clipped-surrogate /
//     value / entropy loss gradients per row, then the backward pass;
//   * weight gradients are accumulated in REGISTERS: every thread owns up to 4 4x4 tiles of
//     [dout, din+1] (bias column included) and adds delta^T x over the chunk rows with float4 LDS
//     reads; the same thread applies the Adam update of its tiles (moments in the optimiser's
//     slabs, L2-resident) (optional global-norm clip first) straight into the LDS weights;
//   * a backward phase computes, for one layer, both its weight-gradient accumulation and its input
//     gradient (into a ping-pong LDS buffer), so each layer costs one barrier;
// At the end weights, Adam moments, the last minibatch's gradients and the optimiser step counter
// are written back to the FlatOptimizer slabs.
#include "common.h"
#include "ppo_train.h"

namespace srl {

__device__ __forceinline__ float pt_act(float z, int act) {
  switch (act) {
    case ACT_TANH: return tanhf(z);
    case ACT_RELU: return z > 0.f ? z : 0.f;
    case ACT_ELU: return z > 0.f ? z : expm1f(z);
    default: return z;
  }
}

// activation derivative from the activation OUTPUT y
__device__ __forceinline__ float pt_dact(float y, int act) {
  switch (act) {
    case ACT_TANH: return 1.f - y * y;
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_ELU: return y > 0.f ? 1.f : y + 1.f;
    default: return 1.f;
  }
}

// y[r][j] = act(sum_k x[r][k] W^T[k][j]) for this wave's rows (wave, wave + 8)
__device__ __forceinline__ void pt_forward(const PTLayer& L, float* lds, int lane, int wave) {
  const float* wt = lds + L.wt;
  const float* x0 = lds + L.in_node + wave * L.in_ld;
  const float* x1 = x0 + 8 * L.in_ld;
  float* y0 = lds + L.out_node + wave * L.out_ld;
  float* y1 = y0 + 8 * L.out_ld;
  const int ldw = L.ldw;
  for (int j = lane; j < L.dout; j += 64) {
    float a0 = 0.f, a1 = 0.f, c0 = 0.f, c1 = 0.f;
#pragma unroll 2
    for (int k = 0; k < L.k4; k += 4) {
      const float4 u = *reinterpret_cast<const float4*>(x0 + k);
      const float4 q = *reinterpret_cast<const float4*>(x1 + k);
      const float* wk = wt + k * ldw + j;
      const float w0 = wk[0], w1 = wk[ldw], w2 = wk[2 * ldw], w3 = wk[3 * ldw];
      a0 = fmaf(u.x, w0, a0);
      c0 = fmaf(u.y, w1, c0);
      a0 = fmaf(u.z, w2, a0);
      c0 = fmaf(u.w, w3, c0);
      a1 = fmaf(q.x, w0, a1);
      c1 = fmaf(q.y, w1, c1);
      a1 = fmaf(q.z, w2, a1);
      c1 = fmaf(q.w, w3, c1);
    }
    y0[j] = pt_act(a0 + c0, L.act);
    y1[j] = pt_act(a1 + c1, L.act);
  }
}

// input gradient of layer L for rows (wave, wave + 8): s[r][k] = sum_j d[r][j] W^T[k][j]  (k < din);
// (+ add[r][k]); raw -> dst, else dst = s * act'(y_in).
__device__ __forceinline__ void pt_dx(const PTLayer& L, const float* lds, const float* d, int dld, float* dst, int dst_ld,
                                      const float* add, int add_ld, bool raw, int lane, int wave) {
  const float* wt = lds + L.wt;
  const int jn = L.ldw - 4;  // round4(dout): W^T padding columns are zero
  for (int k = lane; k < L.din; k += 64) {
    const float* wk = wt + k * L.ldw;
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int r = wave + 8 * rr;
      const float* dr = d + r * dld;
      float s0 = 0.f, s1 = 0.f;
#pragma unroll 2
      for (int j = 0; j < jn; j += 4) {
        const float4 dv = *reinterpret_cast<const float4*>(dr + j);
        const float4 wv = *reinterpret_cast<const float4*>(wk + j);
        s0 = fmaf(dv.x, wv.x, s0);
        s1 = fmaf(dv.y, wv.y, s1);
        s0 = fmaf(dv.z, wv.z, s0);
        s1 = fmaf(dv.w, wv.w, s1);
      }
      float s = s0 + s1;
      if (add) s += add[r * add_ld + k];
      if (!raw) s *= pt_dact(lds[L.in_node + r * L.in_ld + k], L.in_act);
      dst[r * dst_ld + k] = s;
    }
  }
}

// one backward phase of layer l: accumulate its weight-gradient tiles (delta^T x over the chunk rows)
// and write its input gradient; one barrier.
__device__ __forceinline__ void pt_phase(const PTArgs& p, float* lds, float (&acc)[PT_MAXT][16], const int (&tl)[PT_MAXT],
                                         const int (&tj0)[PT_MAXT], const int (&tk0)[PT_MAXT], int l, const float* d,
                                         int dld, float* dst, const float* add, bool raw, bool do_dx, int lane, int wave) {
  const PTLayer& L = p.L[l];
#pragma unroll
  for (int i = 0; i < PT_MAXT; ++i) {
    if (tl[i] != l) continue;
    const float* xin = lds + L.in_node + tk0[i];
    const float* dd = d + tj0[i];
#pragma unroll 2
    for (int r = 0; r < PT_R; ++r) {
      const float4 dv = *reinterpret_cast<const float4*>(dd + r * dld);
      const float4 xv = *reinterpret_cast<const float4*>(xin + r * L.in_ld);
      acc[i][0] = fmaf(dv.x, xv.x, acc[i][0]);
      acc[i][1] = fmaf(dv.x, xv.y, acc[i][1]);
      acc[i][2] = fmaf(dv.x, xv.z, acc[i][2]);
      acc[i][3] = fmaf(dv.x, xv.w, acc[i][3]);
      acc[i][4] = fmaf(dv.y, xv.x, acc[i][4]);
      acc[i][5] = fmaf(dv.y, xv.y, acc[i][5]);
      acc[i][6] = fmaf(dv.y, xv.z, acc[i][6]);
      acc[i][7] = fmaf(dv.y, xv.w, acc[i][7]);
      acc[i][8] = fmaf(dv.z, xv.x, acc[i][8]);
      acc[i][9] = fmaf(dv.z, xv.y, acc[i][9]);
      acc[i][10] = fmaf(dv.z, xv.z, acc[i][10]);
      acc[i][11] = fmaf(dv.z, xv.w, acc[i][11]);
      acc[i][12] = fmaf(dv.w, xv.x, acc[i][12]);
      acc[i][13] = fmaf(dv.w, xv.y, acc[i][13]);
      acc[i][14] = fmaf(dv.w, xv.z, acc[i][14]);
      acc[i][15] = fmaf(dv.w, xv.w, acc[i][15]);
    }
  }
  if (do_dx) pt_dx(L, lds, d, dld, dst, p.tmp_ld, add, p.tmp_ld, raw, lane, wave);
  __syncthreads();
}

// W^T (bias-augmented) of every layer from the param slab into LDS, reading the slab in order
// (coalesced) and scattering into the transposed layout; non-temporal loads (L1 bypass) so a
// re-stage after another workgroup's (or this workgroup's) slab writes never sees a stale L1 line.
// The padding slots (j >= dout, k > din, k == din without bias) are never written: zero from start.
__device__ void pt_stage(const PTArgs& p, float* lds, int NL) {
  for (int l = 0; l < NL; ++l) {
    const PTLayer& L = p.L[l];
    for (int o = threadIdx.x; o < L.dout * L.din; o += PT_THREADS) {
      const int j = o / L.din, k = o - j * L.din;
      lds[L.wt + k * L.ldw + j] = __builtin_nontemporal_load(p.param + L.pw + o);
    }
    if (L.pb >= 0)
      for (int j = threadIdx.x; j < L.dout; j += PT_THREADS)
        lds[L.wt + L.din * L.ldw + j] = __builtin_nontemporal_load(p.param + L.pb + j);
  }
}

// Grid-wide barrier of the nwg co-resident workgroups (residency checked by the launcher): monotonic counter,
// producer = every wave drains its stores, lane 0 releases at agent scope and arrives; consumer =
// relaxed polls, one agent-scope acquire, then the workgroup barrier (MI355X_MICROARCH.md,
// inter-workgroup visibility).  The poll gives up after ~1 s and flags `err` so a broken launch ends.
__device__ __forceinline__ void pt_grid_barrier(int* bar, int target, float* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1 << 23)) {
        atomicAdd(err, 1.f);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

__global__ void __launch_bounds__(PT_THREADS) ppo_mlp_train_kernel(PTArgs p) {
  __shared__ __attribute__((aligned(16))) float lds[PT_LDS];
  __shared__ float red[PT_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NL = p.ne + p.na + p.nh + p.nc;
  const int wg = blockIdx.x, nwg = p.nwg;
  int bar_target = 0;
  long long pc[4] = {0, 0, 0, 0}, t_mark = 0;
#define PT_MARK(i)                                  \
  do {                                              \
    if (p.prof) {                                   \
      const long long now = clock64();              \
      if ((i) >= 0) pc[(i) < 0 ? 0 : (i)] += now - t_mark; \
      t_mark = now;                                 \
    }                                               \
  } while (0)

  // ---- stage W^T (bias-augmented) into LDS (padding zeroed first), zero the activation arena
  for (int i = tid; i < p.node_lo; i += PT_THREADS) lds[i] = 0.f;
  __syncthreads();
  pt_stage(p, lds, NL);
  for (int i = p.node_lo + tid; i < p.node_hi; i += PT_THREADS) lds[i] = 0.f;
  __syncthreads();
  if (tid < PT_R) {  // constant-1 bias-input columns
    lds[p.L[0].in_node + tid * p.L[0].in_ld + p.D0] = 1.f;
    for (int l = 0; l < NL; ++l) lds[p.L[l].out_node + tid * p.L[l].out_ld + p.L[l].dout] = 1.f;
  }

  // ---- gradient tiles owned by this thread, their Adam moments
  int tl[PT_MAXT], tj0[PT_MAXT], tk0[PT_MAXT];
  float acc[PT_MAXT][16];
#pragma unroll
  for (int i = 0; i < PT_MAXT; ++i) {
    const int t = tid + i * PT_THREADS;
    tl[i] = -1;
    tj0[i] = tk0[i] = 0;
    for (int l = 0; l < NL; ++l) {
      const PTLayer& L = p.L[l];
      if (t >= L.tile0 && t < L.tile0 + L.tj * L.tk) {
        tl[i] = l;
        tj0[i] = ((t - L.tile0) / L.tk) * 4;
        tk0[i] = ((t - L.tile0) % L.tk) * 4;
      }
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  }
  const float clip = p.clip_p[0], ent = p.ent_p[0];
  float tstep = p.scalars[0];
  float coef = 1.f, norm_last = 0.f;
  float pg_acc = 0.f, v_acc = 0.f, e_acc = 0.f;
  int nsteps = 0;
  const int eh = p.ne + p.na + p.nh - 1;  // head output layer
  const int ec = NL - 1;                  // critic (value) output layer
  const int a0l = p.ne, c0l = p.ne + p.na + p.nh;
  float* TA = lds + p.tmpA;
  float* TB = lds + p.tmpB;
  float* TD = lds + p.tmpD;
  __syncthreads();

  for (int ep = 0; ep < p.epochs; ++ep) {
    const int64_t* perm = p.perm + (size_t)ep * p.n;
    for (int start = 0; start < p.n; start += p.bs) {
      const int Bm = min(p.bs, p.n - start);
      const float invB = 1.f / (float)Bm;
      // the operands of minibatch row `tid` (bs <= PT_THREADS) are fetched once into registers, so
      // no global-memory round trip sits inside the chunk loop
      const bool mine = tid < Bm;
      float robs[PT_MAXD0], ract[PT_MAXA], rlp = 0.f, rvo = 0.f, rret = 0.f, radv = 0.f;
      {
        const int64_t ridx = mine ? perm[start + tid] : 0;
#pragma unroll
        for (int d = 0; d < PT_MAXD0; ++d) robs[d] = (mine && d < p.D0) ? p.obs[ridx * p.D0 + d] : 0.f;
#pragma unroll
        for (int a = 0; a < PT_MAXA; ++a) ract[a] = (mine && a < p.A) ? p.actions[ridx * p.A + a] : 0.f;
        if (mine) {
          rlp = p.logp_old[ridx];
          rvo = p.val_old[ridx];
          rret = p.ret[ridx];
          radv = p.adv[ridx];
        }
      }
      float amean = 0.f, astd = 1.f;
      if (p.norm_adv) {  // (adv - mean) / (std_unbiased + 1e-8) over the minibatch
        amean = block_sum<PT_THREADS / 64>(mine ? radv : 0.f, red) * invB;
        __syncthreads();
        const float d = mine ? radv - amean : 0.f;
        astd = sqrtf(block_sum<PT_THREADS / 64>(d * d, red) / (float)(Bm - 1));
        __syncthreads();
      }
#pragma unroll
      for (int i = 0; i < PT_MAXT; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;

      PT_MARK(-1);
      for (int c0 = wg * PT_R; c0 < Bm; c0 += nwg * PT_R) {
        const int rows = min(PT_R, Bm - c0);
        // ---- observations of the chunk (rows past the minibatch are zero)
        const bool in_chunk = tid >= c0 && tid < c0 + PT_R;
        if (in_chunk) {
          float* o = lds + p.L[0].in_node + (tid - c0) * p.L[0].in_ld;
#pragma unroll
          for (int d = 0; d < PT_MAXD0; ++d)
            if (d < p.D0) o[d] = robs[d];
        }
        __syncthreads();
        // ---- forward: encoder, actor backbone, head, critic (critic[0] reads the features)
        for (int l = 0; l < NL; ++l) {
          pt_forward(p.L[l], lds, lane, wave);
          __syncthreads();
        }
        // ---- loss gradients per row (ppo/loss.py: clipped surrogate, value MSE, entropy)
        if (in_chunk) {
          const int r = tid - c0;
          const PTLayer& H = p.L[eh];
          const PTLayer& V = p.L[ec];
          float* z = lds + H.out_node + r * H.out_ld;
          float* vp = lds + V.out_node + r * V.out_ld;
          if (mine) {
            float mx = -INFINITY;
            for (int a = 0; a < p.A; ++a) mx = fmaxf(mx, z[a]);
            float se = 0.f;
            for (int a = 0; a < p.A; ++a) se += __expf(z[a] - mx);
            const float lse = mx + __logf(se);
            float lpn = 0.f, Hn = 0.f, sa = 0.f;
#pragma unroll
            for (int a = 0; a < PT_MAXA; ++a) {
              if (a >= p.A) break;
              const float la = z[a] - lse, pa = __expf(la);
              lpn += ract[a] * la;
              sa += ract[a];
              Hn -= pa * la;
            }
            const float ratio = __expf(lpn - rlp);
            const float advn = p.norm_adv ? (radv - amean) / (astd + 1e-8f) : radv;
            const float pg1 = advn * ratio;
            const float rc = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip);
            const float pg2 = advn * rc;
            const float inr = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
            const float dmin = pg1 < pg2 ? advn : (pg2 < pg1 ? advn * inr : 0.5f * advn * (1.f + inr));
            const float glp = -dmin * ratio * invB;
#pragma unroll
            for (int a = 0; a < PT_MAXA; ++a) {
              if (a >= p.A) break;
              const float la = z[a] - lse, pa = __expf(la);
              z[a] = glp * (ract[a] - pa * sa) + ent * invB * pa * (la + Hn);
            }
            const float vcur = vp[0];
            float pred = vcur, pass = 1.f;
            if (p.clip_vloss) {
              const float dvv = vcur - rvo;
              pred = rvo + fminf(fmaxf(dvv, -clip), clip);
              pass = (dvv >= -clip && dvv <= clip) ? 1.f : 0.f;
            }
            vp[0] = p.vf_coef * 2.f * (pred - rret) * invB * pass;
            pg_acc += -fminf(pg1, pg2) * invB;
            v_acc += (pred - rret) * (pred - rret) * invB;
            e_acc += -Hn * invB;
          } else {
            for (int a = 0; a < p.A; ++a) z[a] = 0.f;
            vp[0] = 0.f;
          }
        }
        __syncthreads();
        // ---- backward: one barrier per layer (weight-grad tiles + input grad into a ping-pong buffer)
        // critic: value -> ... -> critic[0] (raw input grad of the features into TD)
        const float* d = lds + p.L[ec].out_node;
        int dld = p.L[ec].out_ld;
        for (int l = ec; l >= c0l; --l) {
          float* nx = (d == TA) ? TB : TA;
          if (l == c0l) {
            pt_phase(p, lds, acc, tl, tj0, tk0, l, d, dld, TD, nullptr, true, true, lane, wave);
          } else {
            pt_phase(p, lds, acc, tl, tj0, tk0, l, d, dld, nx, nullptr, false, true, lane, wave);
            d = nx;
            dld = p.tmp_ld;
          }
        }
        // head + actor backbone: logits -> ... -> actor[0] (adds the critic's feature grad)
        d = lds + p.L[eh].out_node;
        dld = p.L[eh].out_ld;
        for (int l = eh; l >= a0l; --l) {
          float* nx = (d == TA) ? TB : TA;
          pt_phase(p, lds, acc, tl, tj0, tk0, l, d, dld, nx, l == a0l ? TD : nullptr, false, true, lane, wave);
          d = nx;
          dld = p.tmp_ld;
        }
        // encoder
        for (int l = p.ne - 1; l >= 0; --l) {
          float* nx = (d == TA) ? TB : TA;
          pt_phase(p, lds, acc, tl, tj0, tk0, l, d, dld, nx, nullptr, false, l > 0, lane, wave);
          d = nx;
          dld = p.tmp_ld;
        }
      }
      // ---- optimiser step: optional global-norm clip, Adam / AdamW on the LDS weights
      PT_MARK(0);
      // publish this workgroup's gradient tiles into partial[wg] in flat-slab order
      {
        float* G = p.partial + (size_t)wg * p.nparam;
#pragma unroll
        for (int i = 0; i < PT_MAXT; ++i) {
          if (tl[i] < 0) continue;
          const PTLayer& L = p.L[tl[i]];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int j = tj0[i] + (e >> 2), k = tk0[i] + (e & 3);
            if (j >= L.dout) continue;
            const int o = k < L.din ? L.pw + j * L.din + k : (k == L.din && L.pb >= 0 ? L.pb + j : -1);
            if (o >= 0) G[o] = acc[i][e];
          }
        }
      }
      if (nwg > 1) {
        bar_target += nwg;
        pt_grid_barrier(p.bar, bar_target, p.err);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      PT_MARK(1);
      // optimiser over this workgroup's contiguous slice of the flat slab (coalesced; the slab's
      // alignment padding has zero gradient, so it stays zero): gradient = sum of the workgroups'
      // partials (also stored as the grad slab), optional global-norm clip, Adam / AdamW
      tstep += 1.f;
      const int per = (((p.nparam + nwg - 1) / nwg) + 3) & ~3;
      const int lo = min(p.nparam, wg * per), hi = min(p.nparam, lo + per);
      const float bc1 = 1.f - powf(p.b1, tstep);
      const float bc2s = sqrtf(1.f - powf(p.b2, tstep));
      const float stp = p.lr / bc1;
      const float decay = p.decoupled ? (1.f - p.lr * p.wd) : 1.f;
      const float l2 = p.decoupled ? 0.f : p.wd;
      const bool clipping = p.max_grad_norm > 0.f;
      coef = 1.f;
      float ss = 0.f;
      for (int base = lo + tid; base < hi; base += 8 * PT_THREADS) {
        float g[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int o = base + q * PT_THREADS;
          g[q] = 0.f;
          if (o < hi)
            for (int w = 0; w < nwg; ++w) g[q] += __builtin_nontemporal_load(p.partial + (size_t)w * p.nparam + o);
        }
        if (clipping) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int o = base + q * PT_THREADS;
            if (o < hi) p.grad[o] = g[q];
            ss += g[q] * g[q];
          }
          continue;
        }
        float pw[8], m0[8], v0[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int o = min(base + q * PT_THREADS, hi - 1);
          pw[q] = p.param[o];
          m0[q] = p.m[o];
          v0[q] = p.v[o];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int o = base + q * PT_THREADS;
          if (o >= hi) break;
          const float gr = g[q] + l2 * pw[q];
          const float mk = m0[q] + (1.f - p.b1) * (gr - m0[q]);
          const float vk = v0[q] * p.b2 + (1.f - p.b2) * gr * gr;
          p.param[o] = pw[q] * decay - stp * mk / (sqrtf(vk) / bc2s + p.eps);
          p.m[o] = mk;
          p.v[o] = vk;
          p.grad[o] = g[q];
        }
      }
      if (clipping) {
        ss = block_sum<PT_THREADS / 64>(ss, red);
        if (nwg > 1) {
          if (tid == 0) p.sq[wg] = ss;
          bar_target += nwg;
          pt_grid_barrier(p.bar, bar_target, p.err);
          ss = 0.f;
          for (int w = 0; w < nwg; ++w) ss += __builtin_nontemporal_load(p.sq + w);
        }
        norm_last = sqrtf(ss);
        coef = fminf(p.max_grad_norm / (norm_last + 1e-6f), 1.f);
        for (int base = lo + tid; base < hi; base += 8 * PT_THREADS) {
          float g[8], pw[8], m0[8], v0[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int o = min(base + q * PT_THREADS, hi - 1);
            g[q] = p.grad[o];
            pw[q] = p.param[o];
            m0[q] = p.m[o];
            v0[q] = p.v[o];
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int o = base + q * PT_THREADS;
            if (o >= hi) break;
            const float gr = g[q] * coef + l2 * pw[q];
            const float mk = m0[q] + (1.f - p.b1) * (gr - m0[q]);
            const float vk = v0[q] * p.b2 + (1.f - p.b2) * gr * gr;
            p.param[o] = pw[q] * decay - stp * mk / (sqrtf(vk) / bc2s + p.eps);
            p.m[o] = mk;
            p.v[o] = vk;
          }
        }
      }
      // every workgroup re-stages the updated weights (its own slice and the others') into LDS
      if (nwg > 1) {
        bar_target += nwg;
        pt_grid_barrier(p.bar, bar_target, p.err);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      pt_stage(p, lds, NL);
      __syncthreads();
      PT_MARK(3);
      ++nsteps;
      __syncthreads();
    }
  }

  if (p.prof && wg == 0 && tid == 0)
    for (int i = 0; i < 4; ++i) p.prof[i] = pc[i];
#undef PT_MARK
  // ---- write back: weights, moments and the last gradients are already in the slabs; loss means, step
  {
    const float a = block_sum<PT_THREADS / 64>(pg_acc, red);
    __syncthreads();
    const float b = block_sum<PT_THREADS / 64>(v_acc, red);
    __syncthreads();
    const float c = block_sum<PT_THREADS / 64>(e_acc, red);
    if (tid == 0) {
      const float inv = nsteps > 0 ? 1.f / (float)nsteps : 0.f;
      atomicAdd(p.out_sums + 0, a * inv);
      atomicAdd(p.out_sums + 1, b * inv);
      atomicAdd(p.out_sums + 2, c * inv);
      if (wg == 0) {
        p.scalars[0] = tstep;
        p.scalars[1] = coef;
        if (p.max_grad_norm > 0.f) p.scalars[2] = norm_last;
      }
    }
  }
}

// resets the loss sums and the grid-barrier counter; a kernel rather than hipMemsetAsync so the
// reset is ordered like every other captured kernel inside a hipGraph (see norm.hip: zero2_kernel)
__global__ void ppo_reset_kernel(float* sums, int* bar) {
  if (threadIdx.x < 3) sums[threadIdx.x] = 0.f;
  if (threadIdx.x == 0 && bar) *bar = 0;
}

}  // namespace srl

hipError_t launch_ppo_mlp_train(const srl::PTArgs& p, hipStream_t st) {
  hipLaunchKernelGGL(srl::ppo_reset_kernel, dim3(1), dim3(64), 0, st, p.out_sums, p.nwg <= 1 ? nullptr : p.bar);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (p.nwg <= 1) {
    hipLaunchKernelGGL(srl::ppo_mlp_train_kernel, dim3(1), dim3(srl::PT_THREADS), 0, st, p);
    return hipGetLastError();
  }
  // The workgroups meet at grid barriers, so all nwg must be resident at once.  That is checked here
  // from the occupancy (nwg is a handful on a 256-CU part) and the barrier itself is bounded (it
  // flags `err` and moves on).  A plain launch, not hipLaunchCooperativeKernel: the cooperative
  // launch path creates a queue of its own whose teardown at process exit faults under rocprofv3
  // kernel tracing (profiles/r2_rocprof_exit_crash.md).
  int dev = 0, cus = 0, per_cu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)srl::ppo_mlp_train_kernel, srl::PT_THREADS, 0);
  if (per_cu < 1 || p.nwg > per_cu * cus) return hipErrorCooperativeLaunchTooLarge;
  hipLaunchKernelGGL(srl::ppo_mlp_train_kernel, dim3(p.nwg), dim3(srl::PT_THREADS), 0, st, p);
  return hipGetLastError();
}
