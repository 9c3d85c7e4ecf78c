"""The side streams the step forks work onto, and the one rule that keeps a captured step valid.

The package runs independent work of one step on side streams (the item tower beside the user
tower, TwoTowerModel; one stream per large table's sort + catch-up chain, functions._lookup_lazy;
opt-in weight-gradient branches). Under hipGraph capture every such stream joins the capture by
waiting on a stream already in it. On this ROCm, a stream that joins through a stream which is
itself a fork of the capture origin (a fork of a fork) makes hipStreamEndCapture segfault, even
when every stream is joined back in order -- tools/capture_fork_repro.py reproduces it with plain
torch ops ('chain', 'chain_fresh', 'chain_dj' crash; 'fork_fresh', one level, does not). That
was the core dump of round 4's user-tower stream (the user tower on its own stream forked its
per-table lookup streams from there) and of a data-parallel captured step (RCCL's internal stream
waits on the stream that issues the collective: the item tower's all-reduce bucket and its
sharded-table exchanges were issued from the item tower's side stream).

Rule: work is forked only from a stream that is not itself one of these side streams
(`can_fork`), and collectives issued while a side stream is current run on the step's root
stream (`on_root`): the root waits for the side stream, the collective forks RCCL's stream from
the root (one level), and for a synchronous collective the side stream then waits for the root.
"""
from __future__ import annotations

import contextlib

import torch

_FORKED = set()  # stream identities of the side streams created here
_ROOT = {}       # device index -> the stream the current step's forward ran on (its fork origin)


def _key(s):
    h = getattr(s, 'cuda_stream', None)
    return h if h is not None else ('id', getattr(s, 'stream_id', id(s)), getattr(s, 'device_index', None))


def side_stream(device, priority=0) -> torch.cuda.Stream:
    """A new side stream, registered as one (no further fork from it)."""
    s = torch.cuda.Stream(device=device, priority=priority)
    _FORKED.add(_key(s))
    return s


def is_side(s) -> bool:
    return _key(s) in _FORKED


def can_fork(s=None) -> bool:
    """Work may be forked from stream s (default: the current one): it is not a side stream."""
    if s is None:
        s = torch.cuda.current_stream()
    return not is_side(s)


def set_root(s) -> None:
    """The stream the step's forward forks its towers from (TwoTowerModel.forward)."""
    _ROOT[s.device.index] = s


@contextlib.contextmanager
def on_root(sync=True):
    """Run a collective on the step's root stream when a side stream is current (module doc);
    `sync`: the side stream waits for it afterwards (its result is read there)."""
    if not torch.cuda.is_available():
        yield
        return
    cur = torch.cuda.current_stream()
    root = _ROOT.get(cur.device.index)
    if root is None or not is_side(cur) or root == cur:
        yield
        return
    root.wait_stream(cur)
    with torch.cuda.stream(root):
        yield
    if sync:
        cur.wait_stream(root)
