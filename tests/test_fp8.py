"""fp8 training linears (ops/fp8.py + csrc/kernels/fp8.hip): delayed-scaling bookkeeping, the fused
cast+transpose kernel against torch's own fp8 conversion, and fp8 GEMMs (hipBLASLt via torch._scaled_mm)
against an fp32 reference of the same linear."""
import pytest
import torch

from pytorch_distributedtraining_amd.ops import fp8 as F8
from pytorch_distributedtraining_amd.ops.linear import Linear


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _check_linear(dev, M=256, K=128, N=192, bias=True, tol=0.08):
    torch.manual_seed(0)
    lin = Linear(K, N, bias=bias).to(dev).to(torch.bfloat16)
    ref = torch.nn.Linear(K, N, bias=bias).to(dev)
    with torch.no_grad():
        ref.weight.copy_(lin.weight.float())
        if bias:
            ref.bias.copy_(lin.bias.float())
    x = torch.randn(4, M // 4, K, device=dev)
    dy = torch.randn(4, M // 4, N, device=dev)
    for it in range(3):                               # iteration 0 (current scaling) and delayed-scaling steps
        xb = x.bfloat16().requires_grad_()
        lin.zero_grad()
        with F8.fp8_autocast():
            y = lin(xb)
        y.backward(dy.bfloat16())
        xr = x.clone().requires_grad_()
        ref.zero_grad()
        yr = ref(xr)
        yr.backward(dy)
        assert y.dtype == torch.bfloat16
        assert rel_err(y, yr) < tol, it
        assert rel_err(xb.grad, xr.grad) < tol, it
        assert rel_err(lin.weight.grad, ref.weight.grad) < tol, it
        if bias:
            assert rel_err(lin.bias.grad, ref.bias.grad) < 0.02
    meta = lin.__dict__["_fp8"]
    assert not any(meta.fresh)
    # history holds the measured amax of x / w / dy; scales follow fmax / amax
    amax_x = float(x.abs().max())
    assert abs(float(meta.hist[0].max()) - amax_x) / amax_x < 0.01
    assert abs(float(meta.scale[0]) - F8.E4M3_MAX / float(meta.hist[0].max())) < 1e-3 * float(meta.scale[0])
    assert abs(float(meta.scale[2]) - F8.E5M2_MAX / float(meta.hist[2].max())) < 1e-3 * float(meta.scale[2])


def test_fp8_linear_cpu():
    _check_linear("cpu")


def test_fp8_update_scales_history_cpu():
    m = F8.Fp8Meta("cpu", history=4)
    for a in (2.0, 8.0, 1.0, 1.0, 1.0, 1.0):
        m.cur[0] = a
        m.update(0, 1, 0)
    # 8.0 left the 4-deep window after 4 more pushes
    assert float(m.hist[0].max()) == 1.0
    assert abs(float(m.scale[0]) - F8.E4M3_MAX) < 1e-3
    assert float(m.cur[0]) == 0.0


def test_fp8_off_outside_autocast_cpu():
    lin = Linear(64, 64).bfloat16()
    lin(torch.randn(16, 64).bfloat16())
    assert "_fp8" not in lin.__dict__


@pytest.mark.gpu
@pytest.mark.parametrize("R,C", [(128, 64), (4096, 2048), (640, 192), (384, 256)])
@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_fp8_cast_transpose_gpu(R, C, fmt, dt):
    torch.manual_seed(0)
    x = (torch.randn(R, C, device="cuda") * 3).to(dt)
    x[0, 0] = 1e4                                     # saturates after scaling (SATFINITE, not NaN)
    meta = F8.Fp8Meta("cuda")
    meta.scale[0] = 0.37
    q, qt = F8.cast_transpose(x, meta, 0, fmt)
    fmax = F8._FMT_MAX[fmt]
    ref = (x.float() * 0.37).clamp(-fmax, fmax).to(F8._FMT_DTYPE[fmt])
    assert torch.equal(q.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(qt.view(torch.uint8), ref.t().contiguous().view(torch.uint8))
    assert float(meta.cur[0]) == float(x.float().abs().max())
    # amax-only pass
    meta.cur.zero_()
    a, b = F8.cast_transpose(x, meta, 0, fmt, want_q=False, want_t=False)
    assert a is None and b is None and float(meta.cur[0]) == float(x.float().abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("R,C", [(96 * 1024, 8192), (96 * 1024 + 64, 8192 + 64)])
def test_fp8_cast_transpose_full_grid_production_shape(R, C):
    """The flagship MLP hidden (96 x 1024 tokens x 8192) through the 128 x 128-tile kernel, and the 64 x 64-tile
    kernel at the same scale (dimensions not multiples of 128): every byte of both outputs and the amax."""
    torch.manual_seed(1)
    x = (torch.randn(R, C, device="cuda") * 3).to(torch.bfloat16)
    meta = F8.Fp8Meta("cuda")
    meta.scale[0] = 0.37
    q, qt = F8.cast_transpose(x, meta, 0, 0)
    ref = (x.float() * 0.37).clamp(-F8._FMT_MAX[0], F8._FMT_MAX[0]).to(F8._FMT_DTYPE[0])
    assert torch.equal(q.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(qt.view(torch.uint8), ref.t().contiguous().view(torch.uint8))
    assert float(meta.cur[0]) == float(x.float().abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("bias", [True, False])
def test_fp8_linear_gpu(bias):
    _check_linear("cuda", M=4096, K=1024, N=2048, bias=bias)


@pytest.mark.gpu
def test_fp8_gpt2_trains_like_bf16():
    """A small GPT-2 under fp8_autocast follows the bf16 loss curve (same init, same batches)."""
    from pytorch_distributedtraining_amd.models import build_gpt2

    def run(fp8):
        torch.manual_seed(0)
        with torch.device("cuda"):
            m = build_gpt2("gpt2-tiny", n_embd=256, n_head=2, n_layer=2).bfloat16()
        opt = torch.optim.AdamW(m.parameters(), lr=3e-3)
        g = torch.Generator(device="cuda")
        g.manual_seed(1)
        # learnable streams (next token = previous + stride mod 512, random start / stride per sequence)
        start = torch.randint(0, 512, (8, 8, 1), device="cuda", generator=g)
        stride = torch.randint(1, 4, (8, 8, 1), device="cuda", generator=g)
        data = (start + stride * torch.arange(257, device="cuda")) % 512
        losses = []
        for i in range(30):
            b = data[i % 8]
            with F8.fp8_autocast(enabled=fp8):
                loss = m(b[:, :-1], labels=b[:, 1:])
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
            losses.append(float(loss))
        return losses, m

    l8, m8 = run(True)
    lb, _ = run(False)
    assert "_fp8" in m8.h[0].mlp.c_fc.__dict__
    assert l8[-1] < 0.5 * l8[0], l8
    assert abs(l8[-1] - lb[-1]) < 0.15 * lb[-1], (l8[-1], lb[-1])


def test_trainer_fp8_requires_bf16_gpu_cpu():
    from pytorch_distributedtraining_amd.trainer import StokeOptimizer, Trainer
    with pytest.raises(ValueError):
        Trainer(torch.nn.Linear(16, 16), optimizer=StokeOptimizer(optimizer=torch.optim.AdamW, optimizer_kwargs={}),
                loss=torch.nn.functional.mse_loss, batch_size_per_device=2, gpu=False, fp16=None, fp8=True,
                verbose=False)


@pytest.mark.gpu
def test_trainer_fp8_gpt2_step():
    """Trainer(fp8=True): the model's Linears take the fp8 path inside Trainer.model and training steps run."""
    from pytorch_distributedtraining_amd.models import build_gpt2
    from pytorch_distributedtraining_amd.trainer import StokeOptimizer, Trainer
    torch.manual_seed(0)
    m = build_gpt2("gpt2-tiny", n_embd=256, n_head=2, n_layer=2)
    tr = Trainer(m, optimizer=StokeOptimizer(optimizer=torch.optim.AdamW, optimizer_kwargs={"lr": 1e-3}),
                 loss=lambda out, y: out, batch_size_per_device=4, gpu=True, fp16="bf16", fp8=True, verbose=False)
    x = torch.randint(0, 512, (4, 129), device="cuda")
    losses = []
    for _ in range(3):
        loss = tr.loss(tr.model(x[:, :-1], labels=x[:, 1:]), None)
        tr.backward(loss)
        tr.step()
        losses.append(float(loss.detach()))
    assert "_fp8" in m.h[0].attn.c_attn.__dict__
    assert all(l == l for l in losses) and losses[-1] < losses[0]


def _check_gelu_mlp(dev, M=256, d=128, tol=0.12):   # two e5m2-quantised gradient stages
    from pytorch_distributedtraining_amd.models.gpt2 import MLP, gpt2_config
    torch.manual_seed(0)
    cfg = gpt2_config("gpt2-tiny", n_embd=d, n_head=2)
    mlp = MLP(cfg).to(dev).bfloat16()
    with torch.no_grad():
        mlp.c_fc.bias.normal_(0, 0.5)
        mlp.c_proj.bias.normal_(0, 0.5)
    ref = [p.detach().float().clone().requires_grad_() for p in (mlp.c_fc.weight, mlp.c_fc.bias, mlp.c_proj.weight,
                                                                 mlp.c_proj.bias)]
    x = torch.randn(2, M // 2, d, device=dev)
    dy = torch.randn(2, M // 2, d, device=dev)
    for it in range(3):
        xb = x.bfloat16().requires_grad_()
        mlp.zero_grad()
        with F8.fp8_autocast():
            y = mlp(xb)
        y.backward(dy.bfloat16())
        xr = x.clone().requires_grad_()
        for r in ref:
            r.grad = None
        h = F8._gelu_tanh(torch.nn.functional.linear(xr, ref[0], ref[1]))
        yr = torch.nn.functional.linear(h, ref[2], ref[3])
        yr.backward(dy)
        assert rel_err(y, yr) < tol, it
        assert rel_err(xb.grad, xr.grad) < tol, it
        for got, want in zip((mlp.c_fc.weight, mlp.c_fc.bias, mlp.c_proj.weight, mlp.c_proj.bias), ref):
            assert rel_err(got.grad, want.grad) < tol, (it, got.shape)
    assert "_fp8" in mlp.c_fc.__dict__ and "_fp8" in mlp.c_proj.__dict__


def test_fp8_gelu_mlp_cpu():
    _check_gelu_mlp("cpu")


@pytest.mark.gpu
def test_fp8_gelu_mlp_gpu():
    _check_gelu_mlp("cuda", M=4096, d=1024)


def test_fp8_linear_output_allows_inplace_cpu():
    """Llama rotates q / k in place inside the qkv projection output: the fp8 linear's output must allow it."""
    lin = Linear(64, 192, bias=False).bfloat16()
    x = torch.randn(2, 16, 64).bfloat16().requires_grad_()
    with F8.fp8_autocast():
        y = lin(x)
    y.view(2, 16, 3, 64)[:, :, 0].mul_(2.0)
    y.float().sum().backward()
    assert x.grad is not None and lin.weight.grad is not None


def test_fp8_with_activation_checkpointing_cpu():
    """Checkpointed blocks recompute under the forward's fp8 setting (same saved tensors, same gradients)."""
    from pytorch_distributedtraining_amd.models import build_gpt2

    def grads(ckpt):
        torch.manual_seed(0)
        m = build_gpt2("gpt2-tiny", n_embd=128, n_head=2, n_layer=2, activation_checkpointing=ckpt).bfloat16()
        x = torch.randint(0, 512, (2, 65))
        with F8.fp8_autocast():
            loss = m(x[:, :-1], labels=x[:, 1:])
        loss.backward()
        return m.h[0].mlp.c_fc.weight.grad.float()
    g0, g1 = grads(False), grads(True)
    assert rel_err(g1, g0) < 1e-2
