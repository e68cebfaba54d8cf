"""fp16 AMP semantics on CPU: an overflowed step changes nothing (parameters, moments, step count), as
torch.amp.GradScaler skips optimizer.step() (torch/amp/grad_scaler.py:360), and with sharded gradients
the overflow seen by ONE rank skips the step on EVERY rank (sharded_grad_scaler.py:262-283).
Reference configuration: AMPConfig(init_scale=2**14), FP16Options.amp (Stoke-DDP.py:182-184,247)."""
import pytest
import torch

from dist_utils import run_workers

from pytorch_distributedtraining_amd.optim import FusedAdamW, GradScaler


def _params(seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(37, generator=g)), torch.nn.Parameter(torch.randn(5, 3, generator=g))]


def test_overflow_step_is_a_no_op_and_keeps_step_count():
    ps = _params()
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FusedAdamW(ps, lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
    topt = torch.optim.AdamW(ref, lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
    g = torch.Generator().manual_seed(1)
    for it in range(6):
        grads = [torch.randn(p.shape, generator=g) for p in ps]
        overflow = it in (1, 4)
        for p, r, gr in zip(ps, ref, grads):
            p.grad = gr.clone()
            r.grad = gr.clone()
        found = torch.tensor([1 if overflow else 0], dtype=torch.int32)
        before = [p.detach().clone() for p in ps]
        opt.step(found_inf=found)
        if overflow:
            assert all(torch.equal(a, b) for a, b in zip(before, ps))
        else:
            topt.step()
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p, r, rtol=1e-6, atol=1e-6)
    assert float(opt.state[ps[0]]["step"]) == 4.0 == float(topt.state[ref[0]]["step"])


def _sharded_overflow(rank, world):
    from pytorch_distributedtraining_amd.parallel import Comm
    comm = Comm()
    ps = _params(seed=10 + rank)          # this rank's disjoint shard of the model
    opt = FusedAdamW(ps, lr=1e-2)
    scaler = GradScaler(init_scale=2.0 ** 14, comm=comm, sharded=True)
    out = []
    for it in range(3):
        for p in ps:
            p.grad = torch.full(p.shape, 0.5 * scaler.get_scale())
        if it == 1 and rank == 1:
            ps[1].grad[2, 1] = float("inf")       # only rank 1's shard overflows
        before = [p.detach().clone() for p in ps]
        scaler.unscale_and_clip(ps, max_norm=0.0)
        found = scaler.step(opt)
        scaler.update()
        changed = not all(torch.equal(a, b) for a, b in zip(before, ps))
        out.append((int(found), changed, scaler.get_scale(), float(opt.state[ps[0]]["step"]) if opt.state else 0.0))
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_overflow_on_one_rank_skips_every_rank(world):
    outs = run_workers(_sharded_overflow, world)
    r0 = outs[0]
    assert all(r == r0 for r in outs)
    (f0, c0, s0, n0), (f1, c1, s1, n1), (f2, c2, s2, n2) = r0
    assert (f0, c0, n0) == (0, True, 1.0)
    assert (f1, c1, n1) == (1, False, 1.0)     # skipped everywhere, Adam step count unchanged
    assert s1 == s0 * 0.5                      # backoff on every rank
    assert (f2, c2, n2) == (0, True, 2.0)
