"""Gradient accessor shared by the optimizer and clipping: engines that keep a low-precision flat
gradient next to an fp32 master parameter expose it as ``param._pdt_grad`` (torch forbids a .grad of a
different dtype), everything else uses ``param.grad``.  A master that shadows a low-precision module
parameter (ZeRO compute-copy mode, parallel/zero.py) names it as ``param._pdt_grad_src`` and reads
that parameter's current ``.grad``."""


def grad_of(p):
    g = getattr(p, "_pdt_grad", None)
    if g is not None:
        return g
    src = getattr(p, "_pdt_grad_src", None)
    if src is not None:
        return src.grad
    return p.grad
