"""Phase timeline of the persistent imagination rollout (csrc/imagine.hip) at the Atari-100k shapes.

Block 0 stamps every hand-off (s_memrealtime, 100 MHz): when its work for the phase was done and when
the row block's NB workgroups had all arrived.  Prints mean work / wait time per phase kind and the
event-timed call, next to the per-op rollout it replaces.

    python scripts/imagine_phases.py [--M 1024] [--horizon 15]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=1024)
    ap.add_argument("--horizon", type=int, default=15)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from test_imagine_gpu import _models

    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.ops import imagine as im

    rssm, actor = _models(512, 512, 512, 512, 2, [9])
    M, S, Hz = a.M, 1024, a.horizon
    post = torch.nn.functional.one_hot(torch.randint(0, 32, (M, 32), device="cuda"), 32).float().view(M, S)
    h = torch.randn(M, 512, device="cuda")

    def timed(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    rssm.fused_imagine = True
    fused = timed(lambda: rssm.imagine_discrete(post, h, actor, Hz))
    rssm.fused_imagine = False
    per_op = timed(lambda: rssm.imagine_discrete(post, h, actor, Hz))
    rssm.fused_imagine = True
    print(f"rollout M={M} H={Hz}: persistent {fused:.3f} ms, per-op {per_op:.3f} ms")

    plan = im._plan(rssm, actor, M)
    La = plan.La
    per_step = La + 5
    n_arr = Hz * per_step + La
    prof = torch.zeros(4096 + 4 * n_arr + 8, dtype=torch.int64, device="cuda")
    ops._ext().set_imagine_prof(prof)
    rssm.imagine_discrete(post, h, actor, Hz)
    torch.cuda.synchronize()
    ops._ext().set_imagine_prof(None)
    ts = prof.cpu().tolist()
    kinds = [f"actor{l}" for l in range(La)] + ["rec", "gx", "h'", "trans1", "trans2"]
    work = {k: [] for k in kinds}
    wait = {k: [] for k in kinds}
    prev = None
    for k in range(n_arr):
        kind = kinds[k % per_step] if k < Hz * per_step else f"actor{k - Hz * per_step}"
        done, ready = ts[2 * k], ts[2 * k + 1]
        if prev is not None:
            work[kind].append((done - prev) / 100.0)  # us (100 MHz)
        wait[kind].append((ready - done) / 100.0)
        prev = ready
    total = (ts[2 * n_arr - 1] - ts[0]) / 100.0
    print(f"block 0 first hand-off -> last: {total:.1f} us ({total / Hz:.1f} us/step)")
    print("phase     work(us)  wait(us)   (means; 'work' of a phase includes the head sampling for rec)")
    for k in kinds:
        wk = sum(work[k]) / max(1, len(work[k]))
        wt = sum(wait[k]) / max(1, len(wait[k]))
        print(f"{k:8s} {wk:9.2f} {wt:9.2f}")
    # sub-phase marks (relative to the previous hand-off's wait-done): rec = [head GEMM start, end,
    # gather start, end]; trans2 = [GEMM start, end, sampled]
    for kind, off in (("rec", La), ("trans2", La + 4)):
        rows = []
        for t in range(Hz):
            k = t * per_step + off
            base = ts[2 * k - 1]
            m = ts[4096 + 4 * k: 4096 + 4 * k + 4]
            rows.append([(x - base) / 100.0 if x else float("nan") for x in m])
        mean = [sum(r[j] for r in rows) / len(rows) for j in range(4)]
        print(f"{kind} sub-phase marks (us from phase start): " + ", ".join(f"{v:.2f}" for v in mean))



if __name__ == "__main__":
    main()
