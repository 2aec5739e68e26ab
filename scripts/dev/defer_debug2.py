import torch
from tests.test_dv3_step_oracle_gpu import _build, _data, _state
from sheeprl_prey_amd.ops import sidestream

tr, opts, moments = _build([9])
data = _data([9])
tr.update_target(1.0)
snap = {k: v.detach().clone() for k, v in _state(tr, opts, moments).items()}
names = [n for n, p in tr.world_model.named_parameters() if p.requires_grad]
params = [p for n, p in tr.world_model.named_parameters() if p.requires_grad]
def restore():
    for k, v in _state(tr, opts, moments).items():
        v.copy_(snap[k])
res = {}
for name, en in (("off", False), ("on", True)):
    restore()
    sidestream.ENABLED = en
    tr.graphed.enabled = False
    torch.cuda.manual_seed(5)
    tr._phase_wm(data)
    torch.cuda.synchronize()
    sidestream.join()
    torch.cuda.synchronize()
    res[name] = [None if p.grad is None else p.grad.detach().clone() for p in params]
    print(name, "queue", dict(sidestream._queue), "pending", dict(sidestream._pending), flush=True)
for i, n in enumerate(names):
    a, b = res["off"][i], res["on"][i]
    if a is None or b is None:
        print(n, "None", a is None, b is None); continue
    d = float((a - b).abs().max())
    if d > 0:
        print(f"{n:70s} off {float(a.norm()):.4e} on {float(b.norm()):.4e} maxdiff {d:.3e}")
