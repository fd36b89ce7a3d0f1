"""HIP-graph replay of a launch-bound inference forward.

A batch-1 KineT forward (``kinet_amd/models/kinet.py``) issues ~150 small
kernels for ~0.1 ms of device work: eager it is host-bound at ~1 ms.  ``GraphedCall`` records
the whole no-grad forward once per input signature into a ``torch.cuda.CUDAGraph`` (the kinet
kernels are launched through ctypes on torch's current stream, so they are captured like
torch's own) and replays it after copying new inputs into the recorded input buffers.

Contract: the callable must be a pure function of its tensor arguments for a fixed signature
(shapes, dtypes, and any Python-level choice such as the number of tracklet queries); the
outputs are the graph's own buffers, overwritten by the next replay.  Tensor-keyed caches
(``kernels.cached``: padding-mask embeddings) are forced to recompute INSIDE the recording,
so a new mask is re-embedded on every replay instead of reusing the warm-up's value.

Weights: the recording holds the device pointers of the weight casts / packings that
``kernels.cached`` built during warm-up.  ``GraphedCall`` keeps every cache entry alive for
its lifetime (so the allocator cannot hand those buffers to anything else) and, given the
module's parameters and buffers, snapshots their (_version, data_ptr, dtype) at record time,
and, given a ``state_fn``, the module-level state the recorded kernels were chosen by (the
compute dtype of ``set_compute_dtype``, the ``training`` flag that selects the op-for-op path):
a replay after ``load_state_dict``, an optimizer step, ``set_compute_dtype`` or ``train()`` /
``eval()`` raises instead of silently running the stale weights or the wrong kernels.
"""
import torch

from kinet_amd import kernels

__all__ = ['GraphedCall']


class GraphedCall:
    def __init__(self, fn, tensors, warmup=3, params=(), state_fn=None):
        self.fn = fn
        self.params = [p for p in params if p is not None]
        self.state_fn = state_fn
        self.static = [t.detach().clone() for t in tensors]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), torch.no_grad():
            for _ in range(max(1, warmup)):      # weight casts / packings cached outside the graph
                fn(*self.static)
        torch.cuda.current_stream().wait_stream(side)
        for t in self.static:                    # bump _version: input-derived caches miss and
            t.copy_(t.clone())                   # are recomputed inside the recording
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph), torch.no_grad():
            self.out = fn(*self.static)
        self._keep = kernels.cache_values()      # the buffers the graph reads stay allocated
        self._pver = self._param_versions()
        self._state = state_fn() if state_fn is not None else None

    def _param_versions(self):
        return [(p._version, p.data_ptr(), p.dtype) for p in self.params]

    def check_weights(self):
        """RuntimeError when a parameter or buffer, or the recorded module state, changed since
        the recording."""
        if self._param_versions() != self._pver:
            raise RuntimeError('GraphedCall: the module parameters changed after the recording '
                               '(load_state_dict / optimizer step); the graph would replay '
                               'the old weights -- record a new GraphedCall')
        if self.state_fn is not None and self.state_fn() != self._state:
            raise RuntimeError(f'GraphedCall: the module state changed after the recording '
                               f'({self._state} -> {self.state_fn()}: set_compute_dtype / train() / eval()); '
                               f'the graph would replay the kernels of the old state -- record a new GraphedCall')

    def __call__(self, *tensors):
        if len(tensors) != len(self.static):
            raise ValueError(f'GraphedCall: {len(tensors)} inputs, recorded with {len(self.static)}')
        for s, t in zip(self.static, tensors):
            if s.shape != t.shape or s.dtype != t.dtype:
                raise ValueError(f'GraphedCall: input {tuple(t.shape)} {t.dtype} does not match the recorded '
                                 f'{tuple(s.shape)} {s.dtype}; record another GraphedCall for this signature')
            s.copy_(t)
        self.check_weights()
        self.graph.replay()
        return self.out
