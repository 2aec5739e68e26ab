import torch
from tests.test_dv3_step_oracle_gpu import _build, _data, _state
from sheeprl_prey_amd.ops import sidestream

tr, opts, moments = _build([9])
data = _data([9])
tr.update_target(1.0)
snap = {k: v.detach().clone() for k, v in _state(tr, opts, moments).items()}
def restore():
    for k, v in _state(tr, opts, moments).items():
        v.copy_(snap[k])
res = {}
for name, en in (("off1", False), ("off2", False), ("on1", True), ("on2", True), ("off3", False)):
    restore()
    sidestream.ENABLED = en
    tr.graphed.enabled = False
    torch.cuda.manual_seed(5)
    out = tr.train_step(data)
    torch.cuda.synchronize()
    o = opts[0]
    per = []
    for i, (p, off) in enumerate(zip(o.params, o.offsets)):
        per.append(float(o.exp_avg[off:off + p.numel()].norm()))
    res[name] = (float(out["Grads/world_model"]), float(out["Loss/world_model_loss"]), per)
    print(name, res[name][0], res[name][1], flush=True)
names = [n for n, _ in tr.world_model.named_parameters() if _.requires_grad]
base = res["off1"][2]
for k in ("off2", "on1", "on2", "off3"):
    bad = [(names[i] if i < len(names) else i, base[i], res[k][2][i]) for i in range(len(base)) if abs(base[i] - res[k][2][i]) > 1e-6 * (abs(base[i]) + 1e-12)]
    print(k, "differing params:", len(bad))
    for b in bad[:15]:
        print("   ", b)
