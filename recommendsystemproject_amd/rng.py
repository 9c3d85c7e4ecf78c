"""Device-resident dropout RNG state ({seed, call counter}, int64[2]).

Seeds are derived from torch.initial_seed() and a per-module counter WITHOUT drawing from torch's
generator, so building our modules consumes exactly the random numbers the reference's
constructors do (identical initial weights under the same torch.manual_seed).
"""
import itertools

import torch

_counter = itertools.count()


def new_rng_state() -> torch.Tensor:
    seed = (torch.initial_seed() * 0x9E3779B1 + 0x632BE5AB * next(_counter)) & 0x7FFFFFFFFFFFFFFF
    return torch.tensor([seed, 0], dtype=torch.int64)
