"""Config dataclass -- field-for-field the reference's `config/config.py:7-67` (names,
defaults and order), so pickled configs in reference checkpoints map onto it and every
field the hot path reads (feature_dim, time_embed_dim, global_points, num_timesteps, schedule,
cond_drop_prob, lambda_chamfer, use_amp, use_hierarchical, ...) means the same thing.

Three additions, keyword fields with defaults that keep the reference behaviour:
`precision` ("fp32": exact-f32 MFMA, the parity default; "bf16": bf16 MFMA perf mode of the
noise MLP, what bench.py measures),
`amp_dtype` (the 16-bit operand format of the training GEMMs under `use_amp`: "float16", the
reference's CUDA autocast default, trainer.py:50,78, or "bfloat16"; same MFMA rate) and
`make_dirs` (the reference creates log/result/checkpoint directories in the CWD on
construction, config.py:64-67; set False to skip)."""
from dataclasses import dataclass
import os


@dataclass
class Config:
    # experiment
    experiment_name: str = "train"
    data_root: str = "datasets"
    processed_data_dir: str = os.path.join("datasets", "processed_hierarchical")
    log_dir: str = "logs"
    checkpoint_dir: str = "checkpoints"
    result_dir: str = "results"

    # hierarchy
    total_points: int = 120000
    global_points: int = 30000

    # model
    time_embed_dim: int = 128
    feature_dim: int = 256
    global_feature_dim: int = 256

    # diffusion
    num_timesteps: int = 1000
    beta_schedule: str = "cosine"
    noise_schedule_offset: float = 0.0008

    # training
    num_epochs: int = 200
    learning_rate: float = 1e-4
    weight_decay: float = 1e-4
    ema_decay: float = 0.999
    gradient_clip: float = 1.0

    # classifier-free guidance
    cond_drop_prob: float = 0.1
    guidance_scale: float = 7.5

    # LR schedule
    lr_scheduler: str = "cosine_with_warmup"
    warmup_epochs: int = 20
    min_lr_ratio: float = 0.01

    # batching
    batch_size: int = 1
    num_workers: int = 2
    use_amp: bool = True
    gradient_accumulation_steps: int = 3

    # validation / saving
    val_interval: int = 5
    save_interval: int = 10

    # loss
    loss_scale_factor: float = 1.0
    use_hierarchical: bool = True
    lambda_chamfer: float = 0.1
    chamfer_loss_on_full_points: bool = False

    # MI355X build additions
    precision: str = "fp32"
    amp_dtype: str = "float16"
    make_dirs: bool = True

    def __post_init__(self):
        if not self.make_dirs:
            return
        exp_checkpoint_dir = os.path.join(self.checkpoint_dir, self.experiment_name)
        for d in [self.log_dir, self.result_dir, self.processed_data_dir, exp_checkpoint_dir]:
            os.makedirs(d, exist_ok=True)

    def __setstate__(self, state):
        # reference pickles carry no `precision` / `amp_dtype` / `make_dirs`: fill the defaults
        self.__dict__.update({"precision": "fp32", "amp_dtype": "float16", "make_dirs": True})
        self.__dict__.update(state)
