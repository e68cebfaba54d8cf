"""fp16 AMP through the Trainer facade on the GPU (fused unscale/clip + fused AdamW, device-side found_inf
and step count) against torch.amp.GradScaler + torch.optim.AdamW, with an injected overflow step.
Reference: AMPConfig(init_scale=2**14) / FP16Options.amp (Stoke-DDP.py:182-184,247), AdamW settings
Stoke-DDP.py:226-235."""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(64, 128), nn.GELU(), nn.Linear(128, 32))


def test_trainer_fp16_amp_matches_torch_gradscaler():
    from pytorch_distributedtraining_amd.trainer import AMPConfig, StokeOptimizer, Trainer

    dev = torch.device("cuda", 0)
    kw = {"lr": 1e-3, "betas": (0.9, 0.99), "eps": 1e-8, "weight_decay": 1e-4}
    ref = _model().to(dev)
    ours = copy.deepcopy(ref)
    tr = Trainer(ours, StokeOptimizer(optimizer=torch.optim.AdamW, optimizer_kwargs=kw), nn.functional.mse_loss,
                 batch_size_per_device=16, gpu=True, fp16="amp", configs=[AMPConfig(init_scale=2 ** 14)],
                 verbose=False)
    topt = torch.optim.AdamW(ref.parameters(), **kw)
    scaler = torch.amp.GradScaler("cuda", init_scale=2 ** 14)
    g = torch.Generator(device=dev).manual_seed(3)
    for it in range(10):
        x = torch.randn(16, 64, device=dev, generator=g)
        y = torch.randn(16, 32, device=dev, generator=g)
        if it == 4:
            x = x * 1e38                          # fp16 overflow inside the autocast region
        loss = tr.loss(tr.model(x), y)
        tr.backward(loss)
        tr.step()
        with torch.autocast("cuda", dtype=torch.float16):
            rl = nn.functional.mse_loss(ref(x), y)
        scaler.scale(rl).backward()
        scaler.step(topt)
        scaler.update()
        topt.zero_grad(set_to_none=True)
        assert tr.scaler.get_scale() == float(scaler.get_scale()), it
    assert tr.scaler.get_scale() == 2 ** 13          # exactly one backoff
    for (n, a), b in zip(ours.named_parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5, msg=n)
    st = tr.optimizer.state[next(ours.parameters())]
    assert float(st["step"]) == 9.0 == float(topt.state[next(ref.parameters())]["step"])
