import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from multimodalreactiongeneration_amd import configs as C
from multimodalreactiongeneration_amd.model import Metaformer
from multimodalreactiongeneration_amd.synthetic import make_batch
from tests.golden_util import rel_err
mc, oc, me = C.lstmformer_config(ratio=1)
torch.manual_seed(0)
m = Metaformer(mc, oc, me).to("cuda:0").eval()
for B, T, lead, devmask in [(3, 40, 4, False), (3, 40, 4, True), (16, 10, 4, True), (37, 25, 12, True), (64, 12, 12, True)]:
    batch = make_batch(B=B, T=T, lead=lead, seed=5, device="cuda:0")
    mask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5)
    if devmask: mask = mask.to("cuda:0")
    with torch.no_grad():
        fast = m._generate(batch, sampling_mask=mask)
    with torch.enable_grad():
        slow = m._generate(batch, sampling_mask=mask).detach()
    torch.cuda.synchronize()
    e = (fast - slow).abs().amax(dim=(0, 2)).cpu()
    print(B, T, lead, devmask, rel_err(fast, slow), "first bad frame", int((e > 1e-5).nonzero()[0]) if (e > 1e-5).any() else None, flush=True)
