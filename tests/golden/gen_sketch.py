"""Gradient sketches shared by the fixture generator (gen_golden.py) and the trainer parity
test: k Rademacher projections of a flattened gradient, the projection matrix regenerated
from the seed (7777, i) for parameter i."""
import numpy as np


def gradient_sketch(g, i, k=32):
    g = np.asarray(g, np.float64).reshape(-1)
    R = np.random.Generator(np.random.PCG64([7777, i])).integers(0, 2, size=(k, g.size)) * 2.0 - 1.0
    return R @ g
