// Parameter block of the persistent RSSM posterior scan (rssm_persist.hip); plain C layout shared
// with the bindings.  Posterior path only: the prior (transition) head does not feed the recurrence,
// so it runs after the scan as batched GEMMs over all T*B rows (ops/rssm.py).
#pragma once

namespace srl {
namespace scanp {

struct PP {
  int T, B, S, D, H, hid, C;
  float alpha, eps1, epsg, eps2;
  int act1, act2;
  int grid;  // workgroups of the launch (every one resident: 1 per CU)
  int offC;  // first workgroup of the forward C phase (categorical tiles)
  int off2;  // first workgroup of the backward G2 / G4 phases
  int ag;    // forward form: 0 = A (gx tiles of 16 columns) -> B (LN-GRU of whole rows + u); 1 = A owns the 16 h
             // columns of all three gates and finishes the LN-GRU of its tile itself (rssm_persist.hip fwd_AG)
  // forward inputs (never written in the launch: plain loads)
  const float *P, *first, *uni, *z0, *Wz, *WzT, *ln1w, *ln1b, *Wg, *lngw, *lngb, *W1, *ln2w, *ln2b, *W2, *b2;
  // forward state: xr holds a_proj + first * (z0 Wz^T) on entry and receives the posterior row gathers
  float *xr, *cat, *zm, *m1, *r1, *gx, *gst, *mg, *rg, *hs, *u, *v, *m2, *r2, *logits, *mixed, *samples;
  int* sel;  // [T][B][S/C] sampled row of Wz^T per (row, categorical), -1 = reset row (hand-off C -> C)
  // backward inputs
  const float *W2T, *W1T, *WgT, *dpost, *dmixed;
  // backward state / outputs: DH holds d_hs on entry, dlog[T-1] is written before the launch
  float *DH, *dlog, *dv, *du, *dgx, *dcat, *dx, *p1g, *p1b, *pgg, *pgb, *p2g, *p2b;
  long ldp;  // row stride of the six LayerNorm parameter partial arrays (column slices of one [T, 2D + 6H + 2hid] buffer)
  // LN-GRU adjoint pieces handed G2 -> G3: dz*gamma per gate column [T][B][3H], row partial sums [T][H/16][16][2]
  float *dZ, *sst;
  // hand-off counters (zeroed before every launch) and the error word (0 = ok)
  unsigned* sync;
  // sticky health word across launches (or-ed with 1 << code on a hand-off timeout; read by the host off
  // the hot path: ops.rssm.check_scan_health) and the spin bound of every wait (0 = default)
  unsigned* health;
  unsigned spin_max;
  // optional phase timestamps (first workgroup of each role, thread 0): prof[(role * T + t) * 8 + k]
  long long* prof;
};

}  // namespace scanp
}  // namespace srl
