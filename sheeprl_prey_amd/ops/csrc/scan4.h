// Parameter block of the 4-launch RSSM scan (rssm_scan.hip); plain C layout shared with the bindings.
#pragma once

namespace srl {
namespace scan4 {

struct SP {
  int T, B, S, D, H, hid, C;
  float alpha, eps1, epsg, eps2;
  int act1, act2;
  // forward inputs
  const float *a_proj, *P, *first, *uni, *z0, *Wz, *ln1w, *ln1b, *Wg, *lngw, *lngb, *W1, *ln2w, *ln2b, *W2, *b2;
  // forward saved / outputs
  float *cat, *zm, *xr, *m1, *r1, *gx, *mg, *rg, *hs, *u, *v, *m2, *r2, *logits, *mixed, *samples;
  // backward
  const float *WzT, *WgT, *W1T, *W2T, *dpost, *dmixed;
  float *DH, *dlog, *dv, *du, *dgx, *dx, *dcat, *dhp, *p1g, *p1b, *pgg, *pgb, *p2g, *p2b;
  // forward: z0 Wz^T (the recurrent input of a reset row), so F4 can fold the one-hot posterior
  // into the next step's recurrent input by row gathers of WzT instead of an F1 GEMM launch
  const float* c0;
  // forward: the posterior's selected WzT row per (step, row, categorical) [T][16][S / C], -1 = none (reset /
  // padding row); F4 of step t writes step t + 1's, FX of step t + 1 gathers them
  int* sel;
  // optional phase timestamps (block 0, thread 0): prof[kernel * 16 + phase] = s_memtime
  long long* prof;
};

}  // namespace scan4
}  // namespace srl
