"""Single-process DDP keeps gradients where autograd puts them (parallel/ddp.py ``_steal_grads``): AccumulateGrad
steals each fresh gradient instead of adding it into a zeroed bucket view.  With fp32 parameters the optimizer
reads the per-parameter gradients; with a bf16 compute copy one multi-tensor gather (queued at the end of every
backward) fills the flat the fp32 masters read.  Checked against a plain module: gradients, accumulation over two
backwards (no_sync), zero_grad, and AdamW steps (FusedAdamW on CPU)."""
import copy
import os

import pytest
import torch
import torch.distributed as dist

from pytorch_distributedtraining_amd.optim import FusedAdamW
from pytorch_distributedtraining_amd.parallel.comm import Comm
from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel


@pytest.fixture(scope="module", autouse=True)
def _pg():
    created = False
    if not dist.is_initialized():
        # file rendezvous: no fixed TCP port to collide with under pytest-xdist
        import tempfile
        d = tempfile.mkdtemp()
        dist.init_process_group("gloo", init_method="file://" + os.path.join(d, "rdzv"), rank=0, world_size=1)
        created = True
    yield
    if created:       # later tests on this worker (fake_world) create their own default group
        dist.destroy_process_group()


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(12, 32), torch.nn.BatchNorm1d(32), torch.nn.ReLU(),
                               torch.nn.Linear(32, 5))


@pytest.mark.parametrize("compute_dtype", [None, torch.bfloat16])
def test_single_process_ddp_steals_gradients(compute_dtype):
    ref = _model()
    ddp = DistributedDataParallel(copy.deepcopy(ref), comm=Comm(), compute_dtype=compute_dtype)
    assert ddp._steal_grads
    if compute_dtype is not None:
        ref = ref.to(compute_dtype)
        for m in ref.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.float()
    xs = [torch.randn(16, 12) for _ in range(2)]
    # two backwards accumulate (the second under no_sync, as a gradient-accumulation micro-step)
    with ddp.no_sync():
        ddp(xs[0].to(compute_dtype or torch.float32)).float().square().mean().backward()
    ddp(xs[1].to(compute_dtype or torch.float32)).float().square().mean().backward()
    for x in xs:
        ref(x.to(compute_dtype or torch.float32)).float().square().mean().backward()
    if compute_dtype is None:
        for p, q in zip(ddp.module.parameters(), ref.parameters()):
            assert p.grad is not None and p.grad._base is None        # autograd's own tensor, not a bucket view
            torch.testing.assert_close(p.grad.float(), q.grad.float(), rtol=1e-2, atol=1e-3)
    else:
        # each backward's stolen gradients were added to the masters' flat and dropped, so every micro-step
        # steals afresh (no per-parameter accumulation adds); the flat holds the accumulated gradient
        assert all(p.grad is None for p in ddp.module.parameters())
        refs = dict(zip(ddp.module.parameters(), ref.parameters()))
        for g in ddp.groups:
            for li, p in enumerate(g.params):
                o = g.offset_of[li]
                torch.testing.assert_close(g.flat_grad[o:o + p.numel()].view_as(p).float(), refs[p].grad.float(),
                                           rtol=2e-2, atol=2e-3)
    opt = FusedAdamW(ddp.optimizer_parameters(), lr=1e-2)
    opt.step()
    opt.zero_grad()
    assert all(p.grad is None for p in ddp.module.parameters())
    if compute_dtype is not None:
        assert all(float(g.flat_grad.abs().sum()) == 0.0 for g in ddp.groups)
    # a second step steals again
    ddp(xs[0].to(compute_dtype or torch.float32)).float().square().mean().backward()
    if compute_dtype is None:
        assert all(p.grad is not None for p in ddp.module.parameters())
    else:
        assert all(float(g.flat_grad.abs().sum()) > 0.0 for g in ddp.groups)
    opt.zero_grad(set_to_none=False)                                   # graph-replay form: zeroed in place
    assert all(p.grad is None or float(p.grad.abs().sum()) == 0.0 for p in ddp.module.parameters())


class _Nested(torch.nn.Module):
    """Returns its prediction nested two levels deep in a dataclass-like object: the master-gradient gather must
    still be queued (only the top level of a tuple/list/dict was searched)."""
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(12, 5)

    def forward(self, x):
        from dataclasses import dataclass

        @dataclass
        class Out:
            extras: dict
        return Out(extras={"aux": [torch.zeros(1), {"pred": self.lin(x)}]})


def test_single_process_ddp_gathers_through_nested_outputs():
    ddp = DistributedDataParallel(_Nested(), comm=Comm(), compute_dtype=torch.bfloat16)
    x = torch.randn(8, 12, dtype=torch.bfloat16)
    out = ddp(x)
    out.extras["aux"][1]["pred"].float().square().mean().backward()
    nz = sum(float(g.flat_grad.abs().sum()) for g in ddp.groups if g.master is not None)
    assert nz > 0, "master gradients stayed zero: the gather was never queued"
