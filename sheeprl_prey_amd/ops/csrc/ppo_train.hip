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

__global__ void __launch_bounds__(PT_THREADS) ppo_mlp_train_kernel(PTArgs p) {
  __shared__ __attribute__((aligned(16))) float lds[PT_LDS];
  __shared__ float red[PT_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NL = p.ne + p.na + p.nh + p.nc;

  // ---- stage W^T (bias-augmented) into LDS, zero the activation arena
  for (int l = 0; l < NL; ++l) {
    const PTLayer& L = p.L[l];
    for (int i = tid; i < L.k4 * L.ldw; i += PT_THREADS) {
      const int k = i / L.ldw, j = i - k * L.ldw;
      float w = 0.f;
      if (j < L.dout) {
        if (k < L.din) w = p.param[L.pw + j * L.din + k];
        else if (k == L.din && L.pb >= 0) w = p.param[L.pb + j];
      }
      lds[L.wt + i] = w;
    }
  }
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

      for (int c0 = 0; c0 < Bm; c0 += PT_R) {
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
      coef = 1.f;
      if (p.max_grad_norm > 0.f) {
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < PT_MAXT; ++i) {
          if (tl[i] < 0) continue;
          const PTLayer& L = p.L[tl[i]];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int j = tj0[i] + (e >> 2), k = tk0[i] + (e & 3);
            if (j < L.dout && (k < L.din || (k == L.din && L.pb >= 0))) ss += acc[i][e] * acc[i][e];
          }
        }
        ss = block_sum<PT_THREADS / 64>(ss, red);
        norm_last = sqrtf(ss);
        coef = fminf(p.max_grad_norm / (norm_last + 1e-6f), 1.f);
      }
      tstep += 1.f;
      const float bc1 = 1.f - powf(p.b1, tstep);
      const float bc2s = sqrtf(1.f - powf(p.b2, tstep));
      const float stp = p.lr / bc1;
      const float decay = p.decoupled ? (1.f - p.lr * p.wd) : 1.f;
      const float l2 = p.decoupled ? 0.f : p.wd;
#pragma unroll
      for (int i = 0; i < PT_MAXT; ++i) {
        if (tl[i] < 0) continue;
        const PTLayer& L = p.L[tl[i]];
        int ot[16];
        float mt[16], vt[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {  // issue all 32 moment loads of the tile before using any
          const int j = tj0[i] + (e >> 2), k = tk0[i] + (e & 3);
          ot[e] = j >= L.dout ? -1 : (k < L.din ? L.pw + j * L.din + k : (k == L.din && L.pb >= 0 ? L.pb + j : -1));
          mt[e] = ot[e] >= 0 ? p.m[ot[e]] : 0.f;
          vt[e] = ot[e] >= 0 ? p.v[ot[e]] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if (ot[e] < 0) continue;
          const int j = tj0[i] + (e >> 2), k = tk0[i] + (e & 3);
          float* w = lds + L.wt + k * L.ldw + j;
          const float pw = *w;
          const float gr = acc[i][e] * coef + l2 * pw;
          const float mk = mt[e] + (1.f - p.b1) * (gr - mt[e]);
          const float vk = vt[e] * p.b2 + (1.f - p.b2) * gr * gr;
          *w = pw * decay - stp * mk / (sqrtf(vk) / bc2s + p.eps);
          p.m[ot[e]] = mk;
          p.v[ot[e]] = vk;
        }
      }
      ++nsteps;
      __syncthreads();
    }
  }

  // ---- write back: weights (LDS -> slab), Adam moments, last gradients, step counter, loss means
  for (int l = 0; l < NL; ++l) {
    const PTLayer& L = p.L[l];
    for (int i = tid; i < L.dout * L.din; i += PT_THREADS) {
      const int j = i / L.din, k = i - j * L.din;
      p.param[L.pw + i] = lds[L.wt + k * L.ldw + j];
    }
    if (L.pb >= 0)
      for (int j = tid; j < L.dout; j += PT_THREADS) p.param[L.pb + j] = lds[L.wt + L.din * L.ldw + j];
  }
#pragma unroll
  for (int i = 0; i < PT_MAXT; ++i) {
    if (tl[i] < 0) continue;
    const PTLayer& L = p.L[tl[i]];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int j = tj0[i] + (e >> 2), k = tk0[i] + (e & 3);
      if (j >= L.dout) continue;
      int o = -1;
      if (k < L.din) o = L.pw + j * L.din + k;
      else if (k == L.din && L.pb >= 0) o = L.pb + j;
      if (o < 0) continue;
      p.grad[o] = acc[i][e];
    }
  }
  {
    const float a = block_sum<PT_THREADS / 64>(pg_acc, red);
    __syncthreads();
    const float b = block_sum<PT_THREADS / 64>(v_acc, red);
    __syncthreads();
    const float c = block_sum<PT_THREADS / 64>(e_acc, red);
    if (tid == 0) {
      const float inv = nsteps > 0 ? 1.f / (float)nsteps : 0.f;
      p.out_sums[0] = a * inv;
      p.out_sums[1] = b * inv;
      p.out_sums[2] = c * inv;
      p.scalars[0] = tstep;
      p.scalars[1] = coef;
      if (p.max_grad_norm > 0.f) p.scalars[2] = norm_last;
    }
  }
}

}  // namespace srl

void launch_ppo_mlp_train(const srl::PTArgs& p, hipStream_t st) {
  hipLaunchKernelGGL(srl::ppo_mlp_train_kernel, dim3(1), dim3(srl::PT_THREADS), 0, st, p);
}
