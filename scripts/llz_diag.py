import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, "distributed_training_amd/compat/shims")
import torch, torch.nn as nn, torch.distributed as dist
from tests._dist_util import free_port, init_pg
from tests.test_gpu_zero import _micro
torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False
dev = torch.device("cuda", 0)
init_pg("nccl", 0, 1, free_port())
import colossalai
from colossalai.booster import Booster
from colossalai.booster.plugin import LowLevelZeroPlugin
from colossalai.nn.optimizer import HybridAdam
lr = 1e-3
torch.manual_seed(0)
model = _micro().to(dev)
ref16 = _micro().to(dev); ref16.load_state_dict(model.state_dict()); ref16 = ref16.half()
master = [p.detach().float().clone().requires_grad_() for p in ref16.parameters()]
ropt = torch.optim.AdamW(master, lr=lr, weight_decay=0.0, foreach=False)
booster = Booster(plugin=LowLevelZeroPlugin(initial_scale=2 ** 5))
crit = nn.CrossEntropyLoss()
bmodel, bopt, bcrit, _, _ = booster.boost(model, HybridAdam(model.parameters(), lr=lr), criterion=crit)
z = bopt.zero
print("hp", z.hp, z.kind, "scale", z.scaler.scale)
names = [n for n, _ in model.named_parameters()]
for it in range(3):
    g = torch.Generator(device=dev).manual_seed(100 + it)
    x = torch.rand(8, 3, 32, 32, device=dev, generator=g)
    y = torch.randint(0, 10, (8,), device=dev, generator=g)
    # forward equality
    with torch.no_grad():
        o1 = bmodel(x); o2 = ref16(x.half()).float()
    print("it", it, "fwd maxdiff", (o1 - o2).abs().max().item())
    loss = bcrit(bmodel(x), y)
    booster.backward(loss, bopt)
    bopt.step(); bopt.zero_grad()
    (crit(ref16(x.half()).float(), y).float() * 32.0).backward()
    with torch.no_grad():
        for m, p in zip(master, ref16.parameters()):
            m.grad = p.grad.float() * (1.0 / 32.0); p.grad = None
    ropt.step()
    with torch.no_grad():
        for m, p in zip(master, ref16.parameters()):
            p.copy_(m.half())
    mine = z.consolidated_state_dict()
    worst = max(((mine[n].to(dev) - m.detach()).abs().max().item(), n) for n, m in zip(names, master))
    print("it", it, "master maxdiff", worst, "scale", z.scaler.scale, "steps", z.step_count)
# fp16 params vs master.half() on our side
mine = z.consolidated_state_dict()
for n, p16 in model.named_parameters():
    m = mine[n].to(dev).float()
    bad = (p16.detach() != m.half())
    if bad.any():
        idx = bad.reshape(-1).nonzero()[:5].reshape(-1)
        print("param16 != master.half()", n, int(bad.sum()), "of", bad.numel(),
              [(float(m.reshape(-1)[i]), float(p16.detach().reshape(-1)[i]), float(m.half().reshape(-1)[i])) for i in idx])
