"""Oracle outputs of the 120k-point guided loop, for the end-to-end gate of the measured mode
(tests/test_gpu_configs.py::test_loop_vs_oracle_50_steps_120k).

The oracle (oracle/oracle.py, itself pinned to the reference by gen_golden.py's fixtures) runs
`guided_sample_loop` (/root/reference/models/diffusion_model.py:224-261) on the lidar-like
120k cloud pair (synthetic.lidar_like_cloud seeds 1000 / 2000), x_T = standard_normal(3000),
deterministic weights (detweights.py), guidance 7.5, counter-keyed draws rng.CounterRNG(6000),
for a 50-step schedule and for BASELINE configs[1]'s full 1000-step schedule (every t; the
headline metric times this schedule).  A 50-step run takes minutes on the host and the
1000-step run ~20 minutes, too long for a GPU test, so the outputs are committed here (float32,
1.4 MB each).

    python tests/golden/gen_oracle_loop.py        # -> tests/golden/oracle_loop120k.npz (x_50)
    python tests/golden/gen_oracle_loop.py 1000   # -> tests/golden/oracle_loop120k_1000.npz
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)


def main():
    from detweights import deterministic_state
    from oracle import oracle as O
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.model_spec import state_dict_shapes
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    sd = deterministic_state(state_dict_shapes())
    src = lidar_like_cloud(1000, 120000)[None]
    cond = lidar_like_cloud(2000, 120000)[None]
    xT = standard_normal(3000, (1, 120000, 3))
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    t0 = time.perf_counter()
    out = {f"x_{S}": O.guided_loop_counter(sd, src, cond, xT, S, rng.CounterRNG(6000))}
    print(f"{S} steps: {time.perf_counter() - t0:.1f} s", flush=True)
    name = "oracle_loop120k.npz" if S == 50 else f"oracle_loop120k_{S}.npz"
    np.savez_compressed(os.path.join(HERE, name), **out)


if __name__ == "__main__":
    main()
