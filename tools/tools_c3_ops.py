"""Which host ops issue the small device copies / fills of the C3 scheduled-sampling step
(torch.profiler over one eager step, grouped by the innermost Python frames).

    python tools/tools_c3_ops.py          (on a GPU box)
"""
import os
import sys

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd.model import LSTMwithSample  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402

DEV = "cuda:0"
mc, oc, me = C.lstm_with_sampling_config(use_scheduled_sampling=True)
torch.manual_seed(0)
m = LSTMwithSample(mc, oc, me).to(DEV)
m.current_epoch = 30
opt = m.configure_optimizers()["optimizer"]
batch = make_batch(B=64, T=300, lead=12, seed=1234, device=DEV)
mask = torch.from_numpy(np.random.RandomState(7).rand(300) < 0.5).to(DEV)


def step():
    opt.zero_grad()
    m.training_step(batch, sampling_mask=mask)["loss"].backward()
    opt.step()


step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="count", row_limit=40))
print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=25, max_name_column_width=60))
