"""HIP-graph replay of a whole training step (forward, loss, backward, fused BertAdam).

At small per-rank batches the MMBT step is bound by the host, not the GPU: ~2,200 kernel
launches per step, each a Python -> ctypes -> hipLaunchKernel round trip, take about as long
to enqueue as the GPU takes to run them (batch 32: host enqueue 35-39 ms against a 38 ms
step, profiles/r3_host_overhead_ab.txt).  Batch 32 is the per-rank batch of BASELINE
config 4 on 8 GPUs (global 256 / 8 ranks).  Capturing the step once into a hipGraph
(torch.cuda.CUDAGraph drives hipStreamBeginCapture / hipGraphLaunch on ROCm) and
replaying it issues the same kernels, in the same order, on the same streams, with one host
call per step.

What a replayable step needs, and where each holds:
* static shapes and buffers: the inputs are the tensors the step was captured with; a caller
  with new data copies it into them (``StepGraph.inputs``) before ``replay()``;
* dropout: the seeds the host draws while capturing (src/mmbt.py ``_seed``) are baked into
  the captured launches.  The graph's first node advances a device counter that every
  dropout kernel folds into its seed when it runs (``kernels.set_seed_offset`` /
  include/mmu.h ``mmu_set_seed_offset``), so each replay draws new masks and the forward
  and backward of one replay agree (they read the same counter value);
* the optimizer: the fused BertAdam keeps its step counts and the warmup_linear schedule on
  the device (csrc/optim.hip), so nothing host-side changes between steps;
* no host synchronisation inside the step (none on the MMBT train path);
* the side stream of the deferred weight gradients joins the capture through the events of
  ``side.wait_stream(main)`` and rejoins the main stream when the backward ends
  (kernels.join_at_backward_end), as eager execution does.

The warmup steps run eagerly on the capture stream first: MIOpen's solver search, the
per-stream split-K workspaces (kernels._splitk_workspace) and every lazily built buffer
exist before capture, and the workspaces keyed by stream are the capture stream's own.
Reference: the step replayed is src/framework.py:276-304 (Model_.train_loop's inner body).
"""
import torch

from . import kernels as K


class StepGraph:
    """Capture ``step_fn`` (no arguments; returns the tensors to keep, e.g. the loss) after
    ``warmup`` eager runs; ``replay()`` runs one more step and returns those tensors (updated
    in place by every replay)."""

    def __init__(self, step_fn, device, warmup=3, inputs=()):
        self.device = torch.device(device)
        self.inputs = tuple(inputs)
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        K.set_seed_offset(self.counter)
        self.stream = torch.cuda.Stream(device=self.device)
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            for _ in range(warmup):
                self.counter.add_(1)
                step_fn()
        cur.wait_stream(self.stream)
        torch.cuda.synchronize(self.device)
        # the warm-up's cached activations go back to the driver: the capture allocates the
        # step's buffers again, in the graph's private pool
        torch.cuda.empty_cache()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            self.counter.add_(1)
            self.out = step_fn()
        torch.cuda.synchronize(self.device)

    def replay(self):
        self.graph.replay()
        return self.out

    def release(self):
        """Drop the graph (its private memory pool returns to the allocator) and the seed counter."""
        K.set_seed_offset(None)
        self.graph.reset()
        self.out = None
