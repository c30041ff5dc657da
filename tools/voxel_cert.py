"""Certified collision-free voxel boxes for the dense voxel grid (csrc/voxel.hip PCST_DENSE_BOXES).

    python tools/voxel_cert.py

The reference groups points by the int32 xor-hash of their voxel coordinates
(models/diffusion_model.py:89-92: (vx*73856093) ^ (vy*19349663) ^ (vz*83492791)), so two voxels
whose hashes collide form one group.  A box [0,X) x [0,Y) x [0,Z) in which all X*Y*Z hashes are
distinct has no such pair, and any box inside it neither.  For each thin extent t of one axis
this prints the largest square cross-section s (box (s, s, t) and its axis permutations) with
distinct hashes, found by bisection (a collision in a box is one in every larger box); the cube
56^3 is collision-free, 60^3 is not.  tests/test_host.py re-checks every box of the table.
A development tool (tools/ only)."""
import numpy as np

PRIMES = (73856093, 19349663, 83492791)


def collision_free(d):
    x = np.arange(d[0], dtype=np.int64)[:, None, None]
    y = np.arange(d[1], dtype=np.int64)[None, :, None]
    z = np.arange(d[2], dtype=np.int64)[None, None, :]
    h = ((x * PRIMES[0]) & 0xFFFFFFFF) ^ ((y * PRIMES[1]) & 0xFFFFFFFF) ^ ((z * PRIMES[2]) & 0xFFFFFFFF)
    h = h.ravel()
    return np.unique(h).size == h.size


def main():
    print("cube 56:", collision_free((56, 56, 56)), " cube 60:", collision_free((60, 60, 60)))
    for thin in (1, 2, 4, 8, 16, 32):
        for ax in range(3):
            def box(s):
                d = [s, s, s]
                d[ax] = thin
                return d
            lo, hi = 1, 1024
            while lo < hi:
                m = (lo + hi + 1) // 2
                if np.prod(box(m)) <= 2 ** 20 and collision_free(box(m)):
                    lo = m
                else:
                    hi = m - 1
            print(thin, ax, box(lo))


if __name__ == "__main__":
    main()
