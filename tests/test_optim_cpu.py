"""FusedAdamW bookkeeping on CPU (advisor round-4 findings):

* per-parameter step counts: the device step counters (``capturable=True`` takes that path on the CPU too) are
  shared only by parameters with identical step histories -- a parameter that receives no gradient on some steps
  keeps its own count, so its bias correction matches torch.optim.AdamW (torch/optim/adam.py:419-547);
* a checkpoint whose parameters carry different step counts loads into per-value counters;
* ``zero_grad`` fills a DDP bucket flat whole only when this optimizer owns every parameter viewing it.
Reference configuration: AdamW(lr=1e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4), Stoke-DDP.py:226-235."""
import copy

import pytest
import torch

from pytorch_distributedtraining_amd.optim import FusedAdamW

KW = dict(lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)


def _pair(seed=0, shapes=((37,), (5, 3), (8,))):
    g = torch.Generator().manual_seed(seed)
    ps = [torch.nn.Parameter(torch.randn(s, generator=g)) for s in shapes]
    return ps, [torch.nn.Parameter(p.detach().clone()) for p in ps]


@pytest.mark.parametrize("capturable", [False, True])
def test_intermittently_unused_parameter_matches_torch(capturable):
    ps, ref = _pair()
    opt = FusedAdamW(ps, capturable=capturable, **KW)
    topt = torch.optim.AdamW(ref, **KW)
    g = torch.Generator().manual_seed(1)
    for it in range(8):
        for i, (p, r) in enumerate(zip(ps, ref)):
            unused = (i == 1 and it % 3 != 0) or (i == 2 and it < 4)     # skips steps / unfrozen late
            gr = None if unused else torch.randn(p.shape, generator=g)
            p.grad = None if gr is None else gr.clone()
            r.grad = None if gr is None else gr.clone()
        opt.step()
        topt.step()
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p, r, rtol=1e-6, atol=1e-6)
    for p, r in zip(ps, ref):
        assert float(opt.state[p]["step"]) == float(topt.state[r]["step"])
    steps = [float(opt.state[p]["step"]) for p in ps]
    assert steps == [8.0, 3.0, 4.0]
    if capturable:
        # the three histories differ: three counters, each owned by one parameter
        assert len(opt._dsteps) == 3


def test_shared_counter_stays_single_while_histories_agree():
    ps, _ = _pair()
    opt = FusedAdamW(ps, capturable=True, **KW)
    for _ in range(3):
        for p in ps:
            p.grad = torch.ones_like(p)
        opt.step()
    assert len(opt._dsteps) == 1
    assert opt.state[ps[0]]["step"] is opt.state[ps[2]]["step"]


def test_checkpoint_with_different_steps_loads_per_value_counters():
    ps, ref = _pair()
    topt = torch.optim.AdamW(ref, **KW)
    g = torch.Generator().manual_seed(3)
    for it in range(5):
        for i, r in enumerate(ref):
            r.grad = None if (i == 0 and it >= 3) else torch.randn(r.shape, generator=g)
        topt.step()
    sd = copy.deepcopy(topt.state_dict())     # a checkpoint, not the live tensors (torch steps them in place)
    for p, r in zip(ps, ref):
        p.data.copy_(r.detach())
    opt = FusedAdamW(ps, capturable=True, **KW)
    opt.load_state_dict(sd)
    for grp in opt.param_groups:
        grp["capturable"] = True                # torch's groups say False: keep the device-counter path
    for it in range(3):
        for p, r in zip(ps, ref):
            gr = torch.randn(p.shape, generator=g)
            p.grad, r.grad = gr.clone(), gr.clone()
        opt.step()
        topt.step()
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p, r, rtol=1e-6, atol=1e-6)
        assert float(opt.state[p]["step"]) == float(topt.state[r]["step"])
    assert len(opt._dsteps) == 2                  # steps 3 (param 0) and 5 (the others), one counter each


def test_zero_grad_fills_a_bucket_flat_only_when_it_owns_every_view():
    a, b = torch.nn.Parameter(torch.zeros(4)), torch.nn.Parameter(torch.zeros(6))
    flat = torch.zeros(10)
    members = [a, b]
    for p, sl in ((a, slice(0, 4)), (b, slice(4, 10))):
        p.grad = flat[sl]
        p._pdt_grad_flat = flat
        p._pdt_grad_members = members
    opt_a, opt_b = FusedAdamW([a], lr=1e-3), FusedAdamW([b], lr=1e-3)
    flat.fill_(1.0)
    opt_a.zero_grad(set_to_none=True)
    assert torch.equal(a.grad, torch.zeros(4)) and a.grad._base is flat        # view kept, zeroed
    assert torch.equal(b.grad, torch.ones(6))                                   # the other optimizer's grads survive
    opt_both = FusedAdamW([a, b], lr=1e-3)
    flat.fill_(2.0)
    opt_both.zero_grad()
    assert torch.equal(flat, torch.zeros(10)) and b.grad._base is flat


@pytest.mark.gpu
def test_device_tables_do_not_pile_up_when_counters_split():
    """tables were keyed by id(counter) and never evicted; a counter split (a parameter skipping steps)
    or a checkpoint reload left dead device tables behind.  Only the live counters' tables stay cached."""
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda")) for s in [(64, 32), (32,), (128,)]]
    opt = FusedAdamW(ps, capturable=True, **KW)
    for it in range(12):
        for i, p in enumerate(ps):
            p.grad = None if (i == 1 and it % 3 != 0) else torch.randn_like(p)
        opt.step()
        assert len(opt._tables) <= len(opt._dsteps)
    sd = copy.deepcopy(opt.state_dict())
    for _ in range(3):                    # repeated reloads: each rebuilds the counters
        opt.load_state_dict(sd)
        for p in ps:
            p.grad = torch.randn_like(p)
        opt.step()
        assert len(opt._tables) <= len(opt._dsteps)


def test_table_cache_retain():
    from pytorch_distributedtraining_amd.ops.multi_tensor import TableCache
    tc = TableCache()
    a, b = torch.zeros(4), torch.zeros(8)
    tc.get((0, "x", 1), [[a]])
    tc.get((0, "x", 2), [[b]])
    tc.get((1, "x", 3), [[b]])
    tc.retain(lambda n: n[0] != 0 or n == (0, "x", 2))
    assert len(tc) == 2
