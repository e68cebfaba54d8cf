"""Gradient accessor shared by the optimizer and clipping: engines that keep a low-precision flat
gradient next to an fp32 master parameter expose it as ``param._pdt_grad`` (torch forbids a .grad of a
different dtype), everything else uses ``param.grad``."""


def grad_of(p):
    g = getattr(p, "_pdt_grad", None)
    return g if g is not None else p.grad
