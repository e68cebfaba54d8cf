#!/usr/bin/env python
"""Why does capturing the SwinIR Trainer step (tests/test_kernels_gpu.py::test_trainer_graph_matches_eager_swinir)
end in a host segfault?  Re-runs that test's setup with torch's sync-debug mode set to "error" for the capture
only: a host synchronisation issued inside the capture then raises with its Python stack instead of crashing."""
import copy
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pytorch_distributedtraining_amd.models.swinir import swinir_s_x2  # noqa: E402
from pytorch_distributedtraining_amd.trainer import ClipGradNormConfig, StokeOptimizer, Trainer  # noqa: E402
from pytorch_distributedtraining_amd.utils import graphs  # noqa: E402

DEV = torch.device("cuda")
orig_graph = torch.cuda.graph


class _strict_graph(orig_graph):
    def __enter__(self):
        r = super().__enter__()
        torch.cuda.set_sync_debug_mode("error")
        return r

    def __exit__(self, *exc):
        torch.cuda.set_sync_debug_mode(0)
        if exc[0] is not None:
            print("EXCEPTION INSIDE CAPTURE:", "".join(traceback.format_exception(*exc)), flush=True)
            os._exit(3)          # do not end the capture (the crash site): report and leave
        return super().__exit__(*exc)


torch.cuda.graph = _strict_graph
torch.manual_seed(0)
base = swinir_s_x2()
g = torch.Generator(device=DEV).manual_seed(3)
data = [(torch.rand(2, 3, 32, 32, device=DEV, generator=g), torch.rand(2, 3, 64, 64, device=DEV, generator=g))
        for _ in range(2)]
opt = StokeOptimizer(optimizer=torch.optim.AdamW, optimizer_kwargs={"lr": 1e-3, "betas": (0.9, 0.99),
                                                                     "eps": 1e-8, "weight_decay": 1e-4})
tr = Trainer(copy.deepcopy(base), optimizer=opt, loss=F.mse_loss, batch_size_per_device=2,
             grad_accum_steps=2, grad_clip=ClipGradNormConfig(max_norm=0.1, norm_type=2.0), gpu=True,
             fp16="bf16", distributed=None, verbose=False)


def step():
    for x, y in data:
        loss = tr.loss(tr.model(x), y)
        tr.backward(loss)
        tr.step()


run = tr.graph(step, warmup=2)
print("capturing", flush=True)
run()
torch.cuda.synchronize()
print("capture + replay ok", flush=True)
