"""HIP-graph capture of a whole training step ("HIP streams and graphs instead of a tracing
compiler").  A step of a fixed-shape model -- forward, backward, gradient clipping coefficient, fused AdamW
-- is a few hundred to a few thousand kernel launches; replaying it as one graph removes the per-launch
host cost (Python dispatch + HIP launch, 5-10 us each), which is what bounds small-batch and many-small-
kernel steps (SwinIR: ~4,600 launches per step).

Requirements on ``step_fn`` (the usual graph-capture rules): static input buffers, no host synchronisation
(``.item()``, ``.cpu()``, data-dependent Python control flow), an optimizer that is capture-safe
(``FusedAdamW(capturable=True)``: device step counter, device clip coefficient), and gradients zeroed in
place (``zero_grad(set_to_none=False)``) so they keep their addresses.

Status: a plain bf16-autocast GPT-2 step (tests/test_kernels_gpu.py::test_graphed_training_step_matches_eager)
and a DistributedDataParallel-wrapped GPT-2 step with a 50,257-row vocabulary
(test_graphed_ddp_gpt2_step_with_large_vocab) replay with losses and weights equal to eager.  The round-1
replay fault (illegal address in a rocprim partition kernel) was torch's embedding dense backward, whose
sort / unique sizes are data-dependent; under capture ``ops.embedding`` uses a fixed-shape HIP scatter-add
instead.  The benchmarked steps are GPU-bound (kernel time ~= step time in the rocprofv3 tables):
``bench.py --workload gpt2-ddp --graph 1`` replays the whole GPT-2 124M step as one graph at 23.26 ms/step vs
23.39 eager (+0.6 %, profiles/r2_gpt2_124m_ddp_graph_ab.log), so the bench default stays eager.

World > 1 (Trainer.graph, ``bench.py --graph 1`` over RCCL): the DDP / ShardedDDP bucket collectives are
captured with the step.  The engines switch to Python post-accumulate readiness hooks first
(``prepare_capture``: the native hooks hold AccumulateGrad nodes bound to the eager stream), the hooks run once
while capturing and the RCCL launches they make are recorded; the xGMI mesh is bypassed while capturing (its
epochs are host-issued kernel arguments).  Pinned on one GPU by
tests/test_kernels_gpu.py::test_graphed_ddp_step_captures_hook_driven_rccl_collectives (a one-rank RCCL group
with the engine's hooks armed as at world 2) and on CPU by the ``capture_safe_hooks`` engine tests.

    step = GraphedStep(train_step, x_static, y_static, warmup=3)
    for x, y in loader:
        loss = step(x, y)        # copies into the static buffers, replays the graph
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GraphedStep:
    """Capture ``step_fn(*static_inputs)`` into a HIP graph on first call and replay it afterwards.

    The first call runs ``warmup`` eager iterations on a side stream (allocator / workspace / kernel-table
    warm-up: these ARE training steps on the first batch), captures one iteration, then replays it -- so the
    first call advances training by ``warmup + 1`` steps and every later call by exactly one."""

    def __init__(self, step_fn: Callable, *static_inputs: torch.Tensor, warmup: int = 3,
                 pool: Optional[tuple] = None):
        if warmup < 1:
            raise ValueError("GraphedStep needs at least one eager warm-up iteration before capture")
        self.fn = step_fn
        self.inputs = static_inputs
        self.warmup = warmup
        self.pool = pool
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None
        self.eager_steps = 0

    def _capture(self):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self.fn(*self.inputs)
                self.eager_steps += 1
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=self.pool):
            self.out = self.fn(*self.inputs)

    def __call__(self, *inputs: torch.Tensor):
        for dst, src in zip(self.inputs, inputs):
            if src is not dst:
                dst.copy_(src, non_blocking=True)
        if self.graph is None:
            self._capture()
        self.graph.replay()
        return self.out

    def reset(self):
        """Drop the captured graph (e.g. after changing the learning rate); the next call re-captures."""
        self.graph = None
        self.out = None
