"""The reference model's parameter/buffer inventory, in state_dict order.

`PointCloudDiffusionModel` (`models/diffusion_model.py:156-163`) registers
style_encoder (PointNet2Encoder sa1/sa2/sa3 conv+BN stacks,
`pointnet2_encoder.py:61-121`, then style_mlp) and noise_predictor
(`diffusion_model.py:38-53`).  80 parameter tensors + 27 buffers; a checkpoint
written by the reference loads into our module tree only if names, order and
shapes agree, which `tests/test_host.py` checks against the recorded manifest.
"""
from __future__ import annotations

SA_LAYOUT = (
    ("sa1", 0, (64, 64, 128)),
    ("sa2", 128, (128, 128, 256)),
    ("sa3", 256, (256, 512, None)),  # None -> feature_dim
)


def state_dict_shapes(feature_dim: int = 256, time_embed_dim: int = 128):
    out = []
    for name, in_ch, mlp in SA_LAYOUT:
        pre = f"style_encoder.encoder.{name}"
        last = in_ch + 3
        chans = [feature_dim if c is None else c for c in mlp]
        for i, c in enumerate(chans):
            out.append((f"{pre}.mlp_convs.{i}.weight", (c, last, 1, 1)))
            out.append((f"{pre}.mlp_convs.{i}.bias", (c,)))
            last = c
        for i, c in enumerate(chans):
            for leaf in ("weight", "bias", "running_mean", "running_var"):
                out.append((f"{pre}.mlp_bns.{i}.{leaf}", (c,)))
            out.append((f"{pre}.mlp_bns.{i}.num_batches_tracked", ()))
    fd = feature_dim
    out += [("style_encoder.style_mlp.0.weight", (512, fd)), ("style_encoder.style_mlp.0.bias", (512,)),
            ("style_encoder.style_mlp.3.weight", (fd, 512)), ("style_encoder.style_mlp.3.bias", (fd,))]
    npd = "noise_predictor"

    def lin(name, o, i):
        out.append((f"{npd}.{name}.weight", (o, i)))
        out.append((f"{npd}.{name}.bias", (o,)))

    lin("point_encoder.0", 128, 3)
    lin("point_encoder.2", 256, 128)
    lin("point_encoder.4", fd, 256)
    lin("time_proj", fd, time_embed_dim)
    lin("style_proj", fd, fd)
    for k in range(6):
        lin(f"layers.{k}.0", 2 * fd, fd)
        lin(f"layers.{k}.2", fd, 2 * fd)
    lin("output_mlp.0", 256, fd)
    lin("output_mlp.2", 128, 256)
    lin("output_mlp.4", 3, 128)
    return out
