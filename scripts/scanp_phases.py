"""Phase timeline of the persistent RSSM scan (csrc/rssm_persist.hip), first workgroup of each role.

Timestamps are s_memrealtime (100 MHz, common to all CUs), so hand-off latencies between roles are
comparable: 'in' = wait for the producers' hand-off, 'prep' = operand staging + LayerNorm/GRU prologue,
'gemm' = register-tile GEMM, 'pub' = epilogue + drain + arrive.

    python scripts/scanp_phases.py        # DreamerV3 Atari-100k shapes: B16 T64 H512 D512 hid512 S1024
"""
import torch

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.dreamer_v3.agent import RSSM, RecurrentModel, init_weights
from sheeprl_prey_amd.models.models import MLP

ROLES = ["A (fwd gx)", "B (fwd GRU/u)", "C (fwd logits)", "G1 (dv)", "G2 (du/DH)", "G3 (dgx/dcat)", "G4 (dx/dlog)"]


def main(H=512, D=512, hid=512, B=16, T=64, E=4096, A=9):
    torch.manual_seed(0)
    S = 32 * 32
    rec = RecurrentModel(S + A, H, D)
    rep = MLP(H + E, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
    tr = MLP(H, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
    rssm = RSSM(rec.apply(init_weights), rep.apply(init_weights), tr.apply(init_weights), {"validate_args": False}).cuda()
    rssm.scan_impl = "persist"
    emb = torch.randn(T, B, E, device="cuda", requires_grad=True)
    act = torch.nn.functional.one_hot(torch.randint(0, A, (T, B), device="cuda"), A).float()
    first = (torch.rand(T, B, 1, device="cuda") < 0.05).float()
    prof = torch.zeros(7 * T * 8, dtype=torch.int64, device="cuda")
    C = ops._ext()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for it in range(4):
        if it == 3:
            C.set_scanp_prof(prof)
        ev[0].record()
        out = rssm.scan_dynamic(emb, act, first)
        ev[1].record()
        sum(o.float().sum() for o in out).backward()
        ev[2].record()
        torch.cuda.synchronize()
    C.set_scanp_prof(None)
    print(f"host-timed scan fwd (+prior head) {ev[0].elapsed_time(ev[1]):.3f} ms, bwd (whole autograd) {ev[1].elapsed_time(ev[2]):.3f} ms")
    p = prof.view(7, T, 8).cpu().double() / 100.0  # us
    for r, name in enumerate(ROLES):
        ts = p[r]
        steps = [t for t in range(T) if ts[t, 0] > 0 and ts[t, 4] > 0]
        if not steps:
            continue
        d = torch.stack([ts[t, 1:5] - ts[t, 0:4] for t in steps])
        per = ts[steps, 4] - ts[steps, 0]
        m = d.mean(0).tolist()
        span = (ts[steps, 4].max() - ts[steps, 0].min()).item()
        print(f"{name:16s} steps {len(steps):3d}  span {span:8.1f} us  per step {per.mean():6.2f} us  "
              f"in {m[0]:5.2f}  prep {m[1]:5.2f}  gemm {m[2]:5.2f}  pub {m[3]:5.2f}")
    # hand-off latency: producer's arrive -> consumer's wait exit, same step
    def lat(prod, cons, shift=0):
        v = [p[cons, t + shift, 1] - p[prod, t, 4] for t in range(T) if 0 <= t + shift < T and p[prod, t, 4] > 0 and p[cons, t + shift, 1] > 0]
        return sum(v) / max(len(v), 1)
    sub = {0: ("xr staged", [(0, 1, 5), (0, 5, 2)]), 1: ("GRU rows done", [(1, 1, 5), (1, 5, 2)]),
           2: ("sampled / C->C in / gathered", [(2, 3, 5), (2, 5, 6), (2, 6, 7), (2, 7, 4)]),
           4: ("dv staged / LN2' regs / partials / finish+du", [(4, 1, 5), (4, 5, 6), (4, 6, 7), (4, 7, 2)]),
           5: ("row stats / dgx / dgx stores", [(5, 1, 5), (5, 5, 6), (5, 6, 2)]),
           6: ("dcat staged / LN1' regs / rest of prep / unimix' / arrive",
               [(6, 1, 5), (6, 5, 6), (6, 6, 2), (6, 3, 7), (6, 7, 4)])}
    for r, (label, pairs) in sub.items():
        vals = []
        for role, k0, k1 in pairs:
            v = [p[role, t, k1] - p[role, t, k0] for t in range(T - 1) if p[role, t, k1] > 0 and p[role, t, k0] > 0]
            vals.append(sum(v) / max(len(v), 1))
        print(f"  {ROLES[r]:16s} sub-phases ({label}): " + "  ".join(f"{x:5.2f}" for x in vals))
    print(f"hand-off A->B {lat(0, 1):.2f} us, B->C {lat(1, 2):.2f} us, C->A(t+1) {lat(2, 0, 1):.2f} us")
    print(f"hand-off G1->G2 {lat(3, 4):.2f} us, G2->G3 {lat(4, 5):.2f} us, G3->G4 {lat(5, 6):.2f} us, G4->G1(t-1) {lat(6, 3, -1):.2f} us")


if __name__ == "__main__":
    main()
