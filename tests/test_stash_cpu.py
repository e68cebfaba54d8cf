"""Column-sum hand-off between backward passes (ops.attention stash / take): the consumer finds what the producer
stashed whether the producer stashed the tensor it returns (a view, whose Python object the autograd engine drops)
or that view's base -- the round-5 bug let every attention backward miss c_proj's colsum(dO) stash."""
import torch

from pytorch_distributedtraining_amd.ops import attention as A


def _chain(stash_returned_view: bool):
    got = {}

    class Consumer(torch.autograd.Function):        # the attention: takes colsum(dO) in its backward
        @staticmethod
        def forward(ctx, x):
            return x.clone().view(2, 4, 2, 3)

        @staticmethod
        def backward(ctx, do):
            got["colsum"] = A.take_dx_colsum(do)
            return do.reshape(2, 4, 6)

    class Producer(torch.autograd.Function):        # the Linear consuming o: stashes db W for its dX
        @staticmethod
        def forward(ctx, y):
            return y * 2

        @staticmethod
        def backward(ctx, dy):
            dx2 = torch.mm(dy.reshape(8, 6), torch.eye(6) * 2)     # a fresh GEMM output (a base)
            dx = dx2.view(*dy.shape)
            A.stash_dx_colsum(dx if stash_returned_view else dx2, torch.arange(6.0))
            return dx

    x = torch.randn(2, 4, 6, requires_grad=True)
    Producer.apply(Consumer.apply(x).reshape(2, 4, 6)).sum().backward()
    return got["colsum"]


def test_stash_on_base_is_taken():
    assert torch.equal(_chain(False), torch.arange(6.0))


def test_stash_on_returned_view_is_taken():
    assert torch.equal(_chain(True), torch.arange(6.0))


def test_stale_stash_is_not_taken():
    """A buffer written in place between stash and take voids the entry (version counter)."""
    g = torch.zeros(8, 6)
    A.stash_bias_grad(g, torch.ones(6))
    g.add_(1.0)
    assert A.take_bias_grad(g) is None
