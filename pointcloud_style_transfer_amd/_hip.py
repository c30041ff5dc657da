"""ctypes binding of libpcst_hip.so (the C ABI declared in include/pcst.h).

This is the only place Python touches the native library.  Every wrapper takes
torch tensors that must live on the HIP device, passes raw device pointers,
shapes and torch's current stream, and raises RuntimeError with
pcst_last_error() on failure.  There is no CPU fallback: a missing library or a
CPU tensor is an error.
"""
from __future__ import annotations

import ctypes
import functools
import os

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# the in-tree library (tools/knobs.py may point an experiment run at another build before the
# first load; the product reads no environment)
LIB_PATH = os.path.join(_HERE, "libpcst_hip.so")

_P = ctypes.c_void_p
_I = ctypes.c_int64
_D = ctypes.c_double
_F = ctypes.c_float
_SZ = ctypes.POINTER(ctypes.c_size_t)

# name -> argtypes (restype int unless listed in _RESTYPES)
SIGNATURES = {
    "pcst_version": [],
    "pcst_last_error": [],
    "pcst_square_distance": [_P, _P, _I, _I, _I, _P, _P],
    "pcst_index_points": [_P, _I, _I, _I, _P, _I, _P, _P],
    "pcst_fps": [_P, _I, _I, _I, _P, _P, _P],
    "pcst_fps_ws": [_P, _I, _I, _I, _P, _P, _P, _P],
    "pcst_fps_workspace_size": [_I, _I, _SZ],
    "pcst_ball_query": [_D, _I, _P, _P, _I, _I, _I, _P, _P],
    "pcst_group_gather": [_P, _P, _I, _I, _I, _P, _P, _I, _I, _P, _P, _P],
    "pcst_voxel_workspace_size": [_I, _I, _SZ],
    "pcst_voxel_stats": [_P, _I, _I, _I, _P, _P, _P],
    "pcst_voxel_select": [_P, _I, _I, _I, _P, _P, _P, _P, ctypes.c_uint64, _P, _P, _P],
    "pcst_voxel_downsample": [_P, _I, _I, _I, _P, ctypes.c_uint64, _P, _P, _P],
    "pcst_voxel_error": [_P, _I, _I, _P, _P],
    "pcst_voxel_copies_workspace_size": [_I, _I, _I, _SZ],
    "pcst_voxel_downsample_copies": [_P, _I, _I, _I, _I, _P, ctypes.c_uint64, _P, _P, _P],
    "pcst_voxel_downsample_copies_prepped": [_P, _I, _I, _I, _I, _P, ctypes.c_uint64, ctypes.c_int,
                                             _P, _P, _P, ctypes.c_uint32, _P],
    "pcst_voxel_downsample_rows": [_P, _I, _I, _I, _I, _P, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                   _P, _P, _P, ctypes.c_uint32, _P, _P, ctypes.c_uint32, _P, _I, _P],
    "pcst_cfg_ddim_voxel_prep": [_P, _P, _P, _I, _I, _F, _F, _F, _F, _F, _P, _P, _P, _I,
                                 ctypes.c_uint64, ctypes.c_int, _P],
    "pcst_knn_workspace_size": [_I, _I, _I, _SZ],
    "pcst_knn3_interp": [_P, _P, _P, _I, _I, _I, _P, _P, _P],
    "pcst_knn3_build": [_P, _P, _I, _I, _I, _I, _I, _P, _P],
    "pcst_cfg_ddim_step_dcoef": [_P, _P, _P, _P, _I, ctypes.c_float, _P, _P, _P, _P],
    "pcst_voxel_downsample_copies_dseed": [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P],
    "pcst_knn3_query": [_P, _P, _I, _I, _I, _P, _P, _P, ctypes.c_uint32, _I, _P],
    "pcst_knn_error": [_P, _I, _I, _I, _P, _P],
    "pcst_knn_stats": [_P, _I, _I, _I, _P, _P],
    "pcst_knn_rows_workspace_size": [_I, _I, _I, _I, _SZ],
    "pcst_knn3_rows_build": [_P, _I, _I, _I, _I, _P, _P, ctypes.c_uint32, _P, ctypes.c_uint32, _P],
    "pcst_knn3_rows_refs": [_P, _P, _I, _I, _I, _I, _P, _P, ctypes.c_uint32, _P, _I, _P],
    "pcst_knn3_rows_query": [_P, _P, _I, _I, _I, _I, _P, _P, _P, ctypes.c_uint32, _P, _I, _P, _I,
                             _P],
    "pcst_knn_rows_stats": [_P, _I, _I, _I, _I, _P, _P],
    "pcst_noise_mlp_blob_bytes": [ctypes.c_int],
    "pcst_noise_cond": [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P],
    "pcst_noise_mlp": [_P, _I, _I, _P, _I, _P, _I, _P, ctypes.c_int, _P, _P],
    "pcst_noise_mlp_ex": [_P, _I, _I, _P, _I, _P, _I, _P, ctypes.c_int, _P, _P, ctypes.c_uint32, _P,
                          _P, ctypes.c_uint32, _P, _P, _I, _P],
    "pcst_cfg_ddim_step": [_P, _P, _P, _P, _I, _F, _F, _F, _F, _F, _P, _P, _P],
    "pcst_pointwise_linear": [_P, _I, _I, _P, _I, _P, _P, ctypes.c_int, _I, _P, _P],
    "pcst_voxel_center_dist": [_P, _I, _P, ctypes.c_float, _P, _P, _P, _P],
    "pcst_knn_dist": [_P, _P, _I, _I, _I, _I, _P, _P, _P],
    "pcst_emd_greedy": [_P, _P, _I, _I, _I, _P, _P],
    "pcst_gemm_nt_bf16": [_P, _I, _I, _P, _I, _P, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "pcst_linear_wgrad_bf16_workspace_size": [_I, _I, _I, _SZ],
    "pcst_linear_wgrad_bf16": [_P, _P, _I, _I, _I, _P, _P, _P, ctypes.c_int, _P],
    "pcst_resblock_fwd16": [_P, _I, _P, _P, _P, _P, ctypes.c_uint64, _F, _P, _P, _P, ctypes.c_int, _P],
    "pcst_cast16_batch": [_P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, _P],
    "pcst_resblock_bwd16": [_P, _I, _P, _P, _P, _P, ctypes.c_uint64, _F, _P, _P, _P, _P, ctypes.c_int, _P],
    "pcst_gemm_ex": [_P, ctypes.c_int, _I, _I, _P, ctypes.c_int, _I, _P, ctypes.c_int,
                     ctypes.c_int, _P, ctypes.c_uint64, _F, _I, _P, _P, ctypes.c_int, _P],
    "pcst_dropout_grad_bf16": [_P, _I, ctypes.c_uint64, _F, _P, ctypes.c_int, _P],
    "pcst_linear_wgrad_ex_workspace_size": [_I, _I, _I, _SZ],
    "pcst_linear_wgrad_ex": [_P, ctypes.c_int, _P, ctypes.c_int, _I, _I, _I, _P, _P, _P,
                             ctypes.c_int, _P],
    "pcst_relu_bwd": [_P, _P, _I, _P, _P],
    "pcst_linear_wgrad_workspace_size": [_I, _I, _I, _SZ],
    "pcst_linear_wgrad": [_P, _P, _I, _I, _I, _P, _P, _P, _P],
    "pcst_channel_stats_workspace_size": [_I, _SZ],
    "pcst_channel_stats": [_P, _I, _I, _P, _P, _P, _P],
    "pcst_affine_act": [_P, _I, _I, _P, _P, ctypes.c_int, _I, _P, _P],
    "pcst_chamfer_fwd_workspace_size": [_I, _I, _I, _SZ],
    "pcst_chamfer_fwd": [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, ctypes.c_int, _P, _P],
    "pcst_chamfer_bwd_workspace_size": [_I, _I, _I, _SZ],
    "pcst_chamfer_bwd": [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "pcst_bn_train_coeffs": [_P, _P, _I, _I, _P, _P, _D, _D, _P, _P, _P, _P, _P, _P],
    "pcst_bn_train_stats": [_P, _I, _I, _P, _P, _D, _D, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "pcst_bn_relu_maxpool": [_P, _I, _I, _P, _P, _I, _P, _P, _P],
    "pcst_bn_relu_bwd_workspace_size": [_I, _SZ],
    "pcst_bn_relu_bwd": [_P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P],
    "pcst_group_gather_bwd_workspace_size": [_I, _I, _SZ],
    "pcst_group_gather_bwd": [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P],
    "pcst_group_colsum16_workspace_size": [_I, _I, _SZ],
    "pcst_group_colsum16": [_P, ctypes.c_int, _I, _I, _I, _P, _P, _P],
    "pcst_l1_workspace_size": [_SZ],
    "pcst_l1_fwd": [_P, _P, _I, _P, _P, _P],
    "pcst_l1_bwd": [_P, _P, _I, _P, _P, _P],
    "pcst_event_create": [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)],
    "pcst_event_destroy": [_P],
    "pcst_event_record": [_P, _P],
    "pcst_stream_wait_event": [_P, _P],
    "pcst_signal_write": [_P, ctypes.c_uint32, _P],
    "pcst_signal_wait": [_P, ctypes.c_uint32, _P, _I, _P],
    "pcst_stream_create": [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)],
    "pcst_stream_destroy": [_P],
    "pcst_event_elapsed_ms": [_P, _P, ctypes.POINTER(ctypes.c_float)],
}
_RESTYPES = {"pcst_version": ctypes.c_char_p, "pcst_last_error": ctypes.c_char_p,
             "pcst_noise_mlp_blob_bytes": ctypes.c_int64}

_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def lib():
    """Load libpcst_hip.so once (fails loudly if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"pcst: {LIB_PATH} not found -- build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(L, name)  # every entry point is exported (tests/test_abi.py)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = L
    return _lib


def version() -> str:
    return lib().pcst_version().decode()


def _call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed ({rc}): {lib().pcst_last_error().decode()}")


def _stream():
    """torch's current stream of the current device.  Every public wrapper runs under
    `_on_tensor_device`, so the current device is the one its tensors live on."""
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _tensor_device_index(args, kwargs):
    """Device index of the first HIP tensor among the arguments (duck-typed), else None."""
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, (tuple, list)):  # knn3_query's (orig, idx, ws) handle
            for b in a:
                if getattr(b, "is_cuda", False):
                    return b.device.index
        elif getattr(a, "is_cuda", False):
            return a.device.index
        elif isinstance(a, KnnRows):
            return a.x.device.index
    return None


def _on_tensor_device(fn):
    """Run a wrapper with the tensors' device current, so the launch goes to that device and
    onto ITS current stream -- also when the caller's current device is another GPU (a model
    on cuda:1 without torch.cuda.set_device)."""
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        idx = _tensor_device_index(args, kwargs)
        if idx is not None and idx != torch.cuda.current_device():
            with torch.cuda.device(idx):
                return fn(*args, **kwargs)
        return fn(*args, **kwargs)

    wrapper.device_guarded = True
    return wrapper


def require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("pcst: tensors must be on the HIP device (cuda); the MI355X "
                               "kernels have no CPU fallback")


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _f32(t):
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


def _i64(t):
    return t.contiguous() if t.dtype == torch.int64 else t.long().contiguous()


# ----------------------------------------------------------------------------- geometry
def square_distance(src, dst):
    require_device(src, dst)
    src, dst = _f32(src), _f32(dst)
    B, S, _ = src.shape
    N = dst.shape[1]
    out = torch.empty(B, S, N, device=src.device, dtype=torch.float32)
    _call("pcst_square_distance", _ptr(src), _ptr(dst), B, S, N, _ptr(out), _stream())
    return out


def index_points(points, idx):
    require_device(points, idx)
    points, idx = _f32(points), _i64(idx)
    B, N = points.shape[:2]
    C = 1
    for d in points.shape[2:]:
        C *= d
    K = idx[0].numel() if idx.dim() > 1 else 1
    out = torch.empty(tuple(idx.shape) + tuple(points.shape[2:]), device=points.device,
                      dtype=torch.float32)
    _call("pcst_index_points", _ptr(points), B, N, C, _ptr(idx), K, _ptr(out), _stream())
    return out


def fps(xyz, npoint, start_idx):
    require_device(xyz, start_idx)
    xyz, start_idx = _f32(xyz), _i64(start_idx)
    B, N, _ = xyz.shape
    out = torch.empty(B, npoint, device=xyz.device, dtype=torch.int64)
    sz = ctypes.c_size_t(0)
    _call("pcst_fps_workspace_size", B, N, ctypes.byref(sz))
    ws = torch.empty(sz.value, device=xyz.device, dtype=torch.uint8) if sz.value else None
    _call("pcst_fps_ws", _ptr(xyz), B, N, npoint, _ptr(start_idx), _ptr(out), _ptr(ws), _stream())
    return out


def ball_query(radius, nsample, xyz, new_xyz):
    require_device(xyz, new_xyz)
    xyz, new_xyz = _f32(xyz), _f32(new_xyz)
    B, N, _ = xyz.shape
    S = new_xyz.shape[1]
    out = torch.empty(B, S, nsample, device=xyz.device, dtype=torch.int64)
    _call("pcst_ball_query", float(radius), nsample, _ptr(xyz), _ptr(new_xyz), B, N, S,
          _ptr(out), _stream())
    return out


def group_gather(xyz, feats, fps_idx, group_idx):
    """Returns (new_xyz [B,S,3], grouped [B,S,ns,3+C])."""
    require_device(xyz, feats, fps_idx, group_idx)
    xyz, fps_idx, group_idx = _f32(xyz), _i64(fps_idx), _i64(group_idx)
    feats = None if feats is None else _f32(feats)
    B, N, _ = xyz.shape
    C = 0 if feats is None else feats.shape[-1]
    S, ns = group_idx.shape[1], group_idx.shape[2]
    new_xyz = torch.empty(B, S, 3, device=xyz.device, dtype=torch.float32)
    grouped = torch.empty(B, S, ns, 3 + C, device=xyz.device, dtype=torch.float32)
    _call("pcst_group_gather", _ptr(xyz), _ptr(feats), B, N, C, _ptr(fps_idx), _ptr(group_idx),
          S, ns, _ptr(new_xyz), _ptr(grouped), _stream())
    return new_xyz, grouped


def _workspace(fn, *dims, device):
    sz = ctypes.c_size_t(0)
    _call(fn, *dims, ctypes.byref(sz))
    return torch.empty(max(sz.value, 1), dtype=torch.uint8, device=device)


# ----------------------------------------------------------------------------- voxel downsample
def voxel_copies_workspace(B, N, copies, device):
    """A workspace for voxel_downsample(..., copies=copies, ws=) of B clouds of N points (zeroed
    once: its pool histogram is kept zero between calls, see cfg_ddim_voxel_prep's pool_seed)."""
    need = ctypes.c_size_t(0)
    _call("pcst_voxel_copies_workspace_size", B, N, copies, ctypes.byref(need))
    return torch.zeros(max(int(need.value), 1), dtype=torch.uint8, device=device)


def voxel_downsample(points, target, seed=0, perm_provider=None, copies=1, ws=None,
                     prepped=False, pool=False, start=None, rows=None, rows_wait=None):
    """HierarchicalProcessor._voxel_grid_downsample_torch for N > target, all clouds at once.

    perm_provider=None: the random subset is drawn on the device from `seed`.
    perm_provider(b, n) -> int64 tensor: replay the reference's torch.randperm(n) for cloud b
    (needs the unique-voxel count, so this path synchronises; used for parity runs).
    copies=k: the result for torch.cat([points] * k) (rows c*B + b) -- on the device-drawn path
    without building or re-hashing the copies (each row keeps the set the concatenated call
    keeps for the same seed); the replay path concatenates, as the reference's draws are per row.
    prepped=True: `ws` was prepared by cfg_ddim_voxel_prep for these points (the device-drawn
    path skips its statistics / zeroing launch); pool=True: that prep also made the pool-key
    histogram for this `seed` (its pool_seed), so the insert skips it.  start (prepped only):
    (flag pointer, value) of a DeviceSignal.next_value() the launch publishes as it begins.
    rows (a KnnRows handle of knn3_rows_build on these clouds, copies and M = target; device-drawn
    path): the emit launch also places the kept points as the handle's refs (phase B,
    pcst_voxel_downsample_rows), so no knn3_rows_refs follows; rows_wait (the build's refs
    DeviceSignal): the placement waits for its last value in-kernel.
    Returns (points [k*B,T,3], idx [k*B,T] int64)."""
    require_device(points)
    points = _f32(points)
    if copies > 1 and perm_provider is not None:
        points = torch.cat([points] * copies)
        copies = 1
    B, N, _ = points.shape
    dev = points.device
    if perm_provider is None:
        if prepped and ws is None:
            raise RuntimeError("voxel_downsample: prepped=True needs the prepared workspace")
        if ws is None:
            ws = voxel_copies_workspace(B, N, copies, dev)
        else:
            need = ctypes.c_size_t(0)
            _call("pcst_voxel_copies_workspace_size", B, N, copies, ctypes.byref(need))
            if ws.numel() < need.value or ws.device != dev:
                raise RuntimeError("voxel_downsample: workspace too small or on another device")
        out_idx = torch.empty(copies * B, target, dtype=torch.int64, device=dev)
        out_pts = torch.empty(copies * B, target, 3, dtype=torch.float32, device=dev)
        if rows is not None:
            if rows.dims != (B, copies, N, target):
                raise RuntimeError(f"voxel_downsample: rows handle {rows.dims} != {(B, copies, N, target)}")
            sflag, sval = start if start is not None else (None, ctypes.c_uint32(0))
            if rows_wait is not None:
                wflag, wval, _, werr, polls = rows_wait.wait_args()
            else:
                wflag, wval, werr, polls = None, ctypes.c_uint32(0), None, ctypes.c_int64(0)
            rows.idx = out_idx
            rows.refs_err = werr
            rows.placed = True
            _call("pcst_voxel_downsample_rows", _ptr(points), B, N, copies, target, _ptr(ws),
                  seed & (2**64 - 1), 1 if prepped else 0, 1 if pool else 0, _ptr(out_idx),
                  _ptr(out_pts), sflag, sval, _ptr(rows.ws), wflag, wval, werr, polls, _stream())
            return out_pts, out_idx
        if prepped:
            sflag, sval = start if start is not None else (None, ctypes.c_uint32(0))
            _call("pcst_voxel_downsample_copies_prepped", _ptr(points), B, N, copies, target,
                  _ptr(ws), seed & (2**64 - 1), 1 if pool else 0, _ptr(out_idx), _ptr(out_pts),
                  sflag, sval, _stream())
        else:
            if start is not None:
                raise RuntimeError("voxel_downsample: start= needs prepped=True")
            if pool:
                raise RuntimeError("voxel_downsample: pool=True needs prepped=True")
            _call("pcst_voxel_downsample_copies", _ptr(points), B, N, copies, target, _ptr(ws),
                  seed & (2**64 - 1), _ptr(out_idx), _ptr(out_pts), _stream())
        return out_pts, out_idx
    ws = _workspace("pcst_voxel_workspace_size", B, N, device=dev)
    out_idx = torch.empty(B, target, dtype=torch.int64, device=dev)
    out_pts = torch.empty(B, target, 3, dtype=torch.float32, device=dev)
    counts = torch.empty(2 * B, dtype=torch.int32, device=dev)
    _call("pcst_voxel_stats", _ptr(points), B, N, target, _ptr(ws), _ptr(counts), _stream())
    c = counts.cpu().tolist()
    perms, offs, lens = [], [], []
    off = 0
    for b in range(B):
        U, P = c[b], c[B + b]
        n = U if U > target else (P if U < target else 0)
        offs.append(off)
        lens.append(n)
        if n:
            p = perm_provider(b, n).to(device=dev, dtype=torch.int64)
            perms.append(p)
            off += n
    perm = torch.cat(perms) if perms else torch.zeros(1, dtype=torch.int64, device=dev)
    offs_t = torch.tensor(offs, dtype=torch.int64, device=dev)
    lens_t = torch.tensor(lens, dtype=torch.int64, device=dev)
    _call("pcst_voxel_select", _ptr(points), B, N, target, _ptr(ws), _ptr(perm), _ptr(offs_t),
          _ptr(lens_t), 0, _ptr(out_idx), _ptr(out_pts), _stream())
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    _call("pcst_voxel_error", _ptr(ws), B, N, _ptr(err), _stream())
    if int(err.item()):
        raise RuntimeError(f"voxel_select: replayed permutation mismatch (code {int(err.item())})")
    return out_pts, out_idx


def voxel_stats(points, target):
    """(U [B], P [B]) on the host -- unique voxels and pool size (diagnostics / tests)."""
    require_device(points)
    points = _f32(points)
    B, N, _ = points.shape
    ws = _workspace("pcst_voxel_workspace_size", B, N, device=points.device)
    counts = torch.empty(2 * B, dtype=torch.int32, device=points.device)
    _call("pcst_voxel_stats", _ptr(points), B, N, target, _ptr(ws), _ptr(counts), _stream())
    c = counts.cpu()
    return c[:B], c[B:]


# ----------------------------------------------------------------------------- kNN upsample
def knn_workspace(B, N, M, device):
    """A workspace for knn3_build/knn3_query (allocate it on the stream that outlives both)."""
    return _workspace("pcst_knn_workspace_size", B, N, M, device=device)


class SignalTimeout(RuntimeError):
    """A device-side wait on a DeviceSignal gave up (the flag's producer never signalled within
    the poll bound): the work ordered behind the wait may have read unfinished data."""


class DeviceSignal:
    """A cross-stream dependency by kernel-side signalling (pcst_signal_write / pcst_signal_wait):
    `signal(stream)` publishes the next value of a device flag after the work enqueued so far on
    `stream`; `wait(stream)` makes `stream`'s later work wait for that value.  Unlike an event
    that another queue waits on, it puts no marker packet on the producer's queue (~3 us there
    instead of ~17 us, tools/sync_probe.hip).  Values grow monotonically; the host holds the
    counter of this flag (no library state).

    A wait that polls `max_polls` times (0: the library's default, ~10 s) without seeing its
    value gives up, sets the flag's error word and lets its stream go on; `check()` (after the
    waiting stream's work) raises SignalTimeout then.  Owners call it once per sampling loop.
    `storage` (optional): an int32 device tensor of 4 elements to live in (so several signals
    can share one allocation and one error read)."""

    # the host counter is passed to the kernels as uint32: a flag retires well before it wraps
    VALUE_LIMIT = 1 << 31

    def __init__(self, device, max_polls=0, storage=None):
        # [flag, timeout error, work-group counter of pcst_noise_mlp_ex's wait, work-group
        #  counter of its start signal (start_all)]
        self.flag = (storage if storage is not None
                     else torch.zeros(4, dtype=torch.int32, device=device))
        if self.flag.dtype != torch.int32 or self.flag.numel() != 4 or not self.flag.is_contiguous():
            raise ValueError("DeviceSignal storage must be 4 contiguous int32")
        self.value = 0
        self.max_polls = int(max_polls)

    def signal(self, stream):
        if self.value + 1 >= self.VALUE_LIMIT:
            raise RuntimeError("DeviceSignal: value would wrap; use a fresh signal")
        self.value += 1
        _call("pcst_signal_write", _ptr(self.flag), self.value, ctypes.c_void_p(stream.cuda_stream))

    def wait(self, stream):
        _call("pcst_signal_wait", _ptr(self.flag), self.value, ctypes.c_void_p(self.flag.data_ptr() + 4),
              self.max_polls, ctypes.c_void_p(stream.cuda_stream))

    def next_value(self):
        """Advance the host counter for a write made by another launch (pcst_noise_mlp_ex's start
        signal): returns (flag pointer, value) to pass to it."""
        if self.value + 1 >= self.VALUE_LIMIT:
            raise RuntimeError("DeviceSignal: value would wrap; use a fresh signal")
        self.value += 1
        return ctypes.c_void_p(self.flag.data_ptr()), ctypes.c_uint32(self.value)

    def wait_args(self):
        """(flag, value, counter, err, max_polls) for pcst_noise_mlp_ex: wait for the last
        signal."""
        base = self.flag.data_ptr()
        return (ctypes.c_void_p(base), ctypes.c_uint32(self.value), ctypes.c_void_p(base + 8),
                ctypes.c_void_p(base + 4), ctypes.c_int64(self.max_polls))

    def timed_out(self) -> bool:
        """Whether any wait on this flag gave up (reads the device: call after the waits ran)."""
        return bool(int(self.flag[1].item()))

    def check(self):
        if self.timed_out():
            raise SignalTimeout("pcst: a cross-stream device wait timed out (its producer never "
                                "signalled); results ordered behind it are invalid")


class DeviceStream:
    """A HIP stream owned by the caller (pcst_stream_create), usable as a torch stream
    (torch.cuda.ExternalStream).  priority < 0: the device's greatest priority."""

    def __init__(self, device, priority=0):
        dev = torch.device(device)
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        h = ctypes.c_void_p()
        with torch.cuda.device(idx):
            _call("pcst_stream_create", int(priority), ctypes.byref(h))
        self._h = h
        self.stream = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))

    def __del__(self):
        try:
            if _lib is not None and self._h:
                _lib.pcst_stream_destroy(self._h)
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass


class DeviceEvent:
    """A stream-ordering event with device-scope fences only (pcst_event_*: hipEventDisableSystemFence).
    The default (torch.cuda.Event) records and waits with system-scope release/acquire, a ~10 us
    bubble per cross-stream dependency in the sampling step; nothing here needs the host to see
    device memory.  timing=True keeps timing (the bench's kernel timing)."""

    def __init__(self, timing=False):
        h = ctypes.c_void_p()
        _call("pcst_event_create", 1 if timing else 0, ctypes.byref(h))
        self._h = h

    def record(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream()
        _call("pcst_event_record", self._h, ctypes.c_void_p(s.cuda_stream))

    def wait(self, stream=None):
        """Make `stream` (default: the current stream) wait for this event."""
        s = stream if stream is not None else torch.cuda.current_stream()
        _call("pcst_stream_wait_event", ctypes.c_void_p(s.cuda_stream), self._h)

    def elapsed_time(self, end):
        ms = ctypes.c_float()
        _call("pcst_event_elapsed_ms", self._h, end._h, ctypes.byref(ms))
        return float(ms.value)

    def __del__(self):
        try:
            if _lib is not None and self._h:
                _lib.pcst_event_destroy(self._h)
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass


def knn3_build(orig, idx, ws=None, lds_floor=0, max_wg=0):
    """Phase 1 of knn3_interp (positions only) on the current stream -> workspace handle
    (orig, idx, workspace) for knn3_query.  `ws` (knn_workspace) may be preallocated, e.g. on
    the stream that runs the query when the build runs on a side stream; `lds_floor` (bytes)
    keeps the build's work-groups off CUs that hold a noise-MLP work-group and `max_wg` caps
    the work-groups of each build launch (pcst.h)."""
    require_device(orig, idx)
    orig, idx = _f32(orig), _i64(idx)
    B, N, _ = orig.shape
    M = idx.shape[1]
    if ws is None:
        ws = _workspace("pcst_knn_workspace_size", B, N, M, device=orig.device)
    _call("pcst_knn3_build", _ptr(orig), _ptr(idx), B, N, M, int(lds_floor), int(max_wg), _ptr(ws),
          _stream())
    return (orig, idx, ws)


def _built_args(built):
    """(flag pointer, value) of the DeviceSignal the build's producer signals, or (NULL, 0)."""
    if built is None:
        return None, 0
    return ctypes.c_void_p(built.flag.data_ptr()), ctypes.c_uint32(built.value)


def knn3_query(coarse, handle, built=None, grid_cap=0):
    """Phase 2 of knn3_interp on the current stream: coarse [B,M,3] -> [B,N,3].  built (the
    DeviceSignal the side-stream build signalled): the query reads the workspace only if that
    flag holds its last value (pcst.h: a timed-out wait then yields eps = 0, reported by the
    signal's error word, instead of a read of a half-built workspace).  grid_cap: at most this
    many query work-groups over all clouds (0: the resident grid; the result never depends on
    it)."""
    orig, idx, ws = handle
    require_device(coarse)
    coarse = _f32(coarse)
    B, N, _ = orig.shape
    M = idx.shape[1]
    if coarse.shape != (B, M, 3):
        raise RuntimeError(f"knn3_query: coarse {tuple(coarse.shape)} != {(B, M, 3)}")
    out = torch.empty(B, N, 3, dtype=torch.float32, device=orig.device)
    _call("pcst_knn3_query", _ptr(coarse), _ptr(orig), B, N, M, _ptr(out), _ptr(ws),
          *_built_args(built), int(grid_cap), _stream())
    return out


def knn3_interp(coarse, orig, idx, check=False, stats=None):
    """HierarchicalProcessor.upsample_knn: coarse [B,M,3], orig [B,N,3], idx [B,M] -> [B,N,3].
    stats (a list): appends {"chunks": [...], "outliers": [...]} per call (diagnostics)."""
    require_device(coarse, orig, idx)
    coarse, orig, idx = _f32(coarse), _f32(orig), _i64(idx)
    B, N, _ = orig.shape
    M = idx.shape[1]
    ws = _workspace("pcst_knn_workspace_size", B, N, M, device=orig.device)
    out = torch.empty(B, N, 3, dtype=torch.float32, device=orig.device)
    _call("pcst_knn3_interp", _ptr(coarse), _ptr(orig), _ptr(idx), B, N, M, _ptr(out), _ptr(ws),
          _stream())
    if check:
        err = torch.zeros(1, dtype=torch.int32, device=orig.device)
        _call("pcst_knn_error", _ptr(ws), B, N, M, _ptr(err), _stream())
        if int(err.item()):
            raise RuntimeError("knn3_interp: coarse index outside [0, N)")
    if stats is not None:
        st = torch.zeros(1 + 2 * B, dtype=torch.int32, device=orig.device)
        _call("pcst_knn_stats", _ptr(ws), B, N, M, _ptr(st), _stream())
        st = st.cpu().tolist()
        stats.append({"chunks": st[1:1 + B], "outliers": st[1 + B:]})
    return out


# kNN-3 upsample, rows layout (pcst_knn3_rows_*): the sampling step's split of the build into
# a positions-only phase over the distinct clouds (beside the voxel downsample) and a one-launch
# ref placement after it.
def knn_rows_workspace(C, copies, N, M, device):
    """A workspace for knn3_rows_build / _refs / _query over C clouds x `copies` CFG rows."""
    return _workspace("pcst_knn_rows_workspace_size", C, copies, N, M, device=device)


class KnnRows:
    """Handle of a rows-layout build: the clouds x [C,N,3], the CFG copies, M and the workspace;
    refs_err: the error word of the ref placement's wait (knn3_rows_refs(wait=...)), which the
    query checks."""

    def __init__(self, x, copies, M, ws):
        self.x, self.copies, self.M, self.ws = x, int(copies), int(M), ws
        self.refs_err = None
        self.placed = False  # the refs were placed by the downsample (voxel_downsample(rows=))

    @property
    def dims(self):
        C, N, _ = self.x.shape
        return C, self.copies, N, self.M


def knn3_rows_build(x, M, copies=1, ws=None, refs_sig=None, done_sig=None):
    """Phase A on the current stream: bin every point of the clouds x [C,N,3] for the query of the
    C * copies CFG rows (row b = cloud b % C) against M refs each -> KnnRows handle.  refs_sig /
    done_sig (DeviceSignals): signalled from this stream once knn3_rows_refs may run (after the
    scan) and once the build is done (after the fill), for work on other streams."""
    require_device(x)
    x = _f32(x)
    C, N, _ = x.shape
    if ws is None:
        ws = knn_rows_workspace(C, copies, N, M, x.device)
    rf, rv = refs_sig.next_value() if refs_sig is not None else (None, ctypes.c_uint32(0))
    df, dv = done_sig.next_value() if done_sig is not None else (None, ctypes.c_uint32(0))
    _call("pcst_knn3_rows_build", _ptr(x), C, int(copies), N, int(M), _ptr(ws), rf, rv, df, dv,
          _stream())
    return KnnRows(x, copies, M, ws)


def knn3_rows_refs(handle, idx, wait=None):
    """Phase B on the current stream (after knn3_rows_build on the handle), one launch: the
    coarse indices idx [C * copies, M] into the rows layout.  wait (a DeviceSignal): the launch
    itself waits for its last signal (phase A on another stream) instead of a wait launch ahead
    of it; a wait that gives up places nothing and sets the signal's error word (its check()
    raises), which the handle's query then also reads (eps = 0, nothing read).  Returns the
    handle."""
    require_device(idx)
    idx = _i64(idx)
    C, copies, N, M = handle.dims
    if tuple(idx.shape) != (C * copies, M):
        raise RuntimeError(f"knn3_rows_refs: idx {tuple(idx.shape)} != {(C * copies, M)}")
    handle.idx = idx  # kept alive until the query
    if wait is not None:
        flag, value, _, err, polls = wait.wait_args()
    else:
        flag, value, err, polls = None, ctypes.c_uint32(0), None, ctypes.c_int64(0)
    handle.refs_err = err
    _call("pcst_knn3_rows_refs", _ptr(handle.x), _ptr(idx), C, copies, N, M, _ptr(handle.ws), flag,
          value, err, polls, _stream())
    return handle


def knn3_rows_query(coarse, handle, built=None, grid_cap=0, waited=False):
    """coarse [C * copies, M, 3] -> [C * copies, N, 3] on the current stream (after
    knn3_rows_refs).  built (the DeviceSignal of the build's done_sig): the query's work-groups
    wait for its last value themselves (a timeout sets its error word and yields eps = 0);
    waited=True: the stream already waited for it (the MLP launch's wait), the work-groups only
    check it; grid_cap as knn3_query."""
    require_device(coarse)
    coarse = _f32(coarse)
    C, copies, N, M = handle.dims
    if tuple(coarse.shape) != (C * copies, M, 3):
        raise RuntimeError(f"knn3_rows_query: coarse {tuple(coarse.shape)} != {(C * copies, M, 3)}")
    out = torch.empty(C * copies, N, 3, dtype=torch.float32, device=coarse.device)
    if built is not None:
        flag, value, _, err, polls = built.wait_args()
        if waited:
            err = None
    else:
        flag, value, err, polls = None, ctypes.c_uint32(0), None, ctypes.c_int64(0)
    _call("pcst_knn3_rows_query", _ptr(coarse), _ptr(handle.x), C, copies, N, M, _ptr(out),
          _ptr(handle.ws), flag, value, err, polls, handle.refs_err, int(grid_cap), _stream())
    return out


def knn_rows_stats(handle):
    """{"err", "chunks" [C], "outliers" [B], "overflow" [B]} of the handle's last build / query
    (synchronises)."""
    C, copies, N, M = handle.dims
    B = C * copies
    st = torch.zeros(1 + C + 2 * B, dtype=torch.int32, device=handle.x.device)
    _call("pcst_knn_rows_stats", _ptr(handle.ws), C, copies, N, M, _ptr(st), _stream())
    st = st.cpu().tolist()
    return {"err": st[0], "chunks": st[1:1 + C], "outliers": st[1 + C:1 + C + B],
            "overflow": st[1 + C + B:]}


def knn3_interp_rows(coarse, x, idx, copies=1):
    """knn3_interp through the rows layout: coarse [C*copies,M,3], the clouds x [C,N,3] (CFG row
    b is cloud b % C), idx [C*copies,M] -> [C*copies,N,3]; the same bits as
    knn3_interp(coarse, cat([x] * copies), idx)."""
    h = knn3_rows_build(x, idx.shape[1], copies)
    knn3_rows_refs(h, idx)
    return knn3_rows_query(coarse, h)


# ----------------------------------------------------------------------------- noise MLP
def noise_mlp_blob_bytes(precision):
    return int(lib().pcst_noise_mlp_blob_bytes(precision))


def noise_cond(t, style, freqs, wt, bt, ws_, bs, b4):
    require_device(t, style)
    t, style = _i64(t), _f32(style)
    C = t.shape[0]
    cond = torch.empty(C, 256, dtype=torch.float32, device=style.device)
    _call("pcst_noise_cond", _ptr(t), _ptr(style), C, _ptr(freqs), _ptr(wt), _ptr(bt), _ptr(ws_),
          _ptr(bs), _ptr(b4), _ptr(cond), _stream())
    return cond


def noise_mlp(pts, points_per_cloud, cond, blob, bias, precision, out=None, wait=None,
              signal=None, signal_all=False):
    """pts [P,3] (P = clouds*points_per_cloud, cloud-major) -> eps [P,3].
    wait (a DeviceSignal signalled on another stream): work queued after the MLP on this stream
    is also ordered after that signal -- at precision 1 (bf16, the solo kernel) by the MLP's
    last work-group (pcst_noise_mlp_ex's wait), otherwise by a wait launch after it.
    signal ((flag, value) from DeviceSignal.next_value()): the value is published as the MLP
    launch begins (everything queued before it on this stream is then done) --
    pcst_noise_mlp_ex's start signal.  signal_all: published once every work-group of the launch
    has begun (the flag's own DeviceSignal storage word 3 counts them: pcst_noise_mlp_ex's
    start_counter), so work another stream starts behind it finds only the CUs the MLP leaves
    idle."""
    require_device(pts, cond, blob, bias)
    pts = _f32(pts)
    P = pts.shape[0]
    if out is None:
        out = torch.empty(P, 3, dtype=torch.float32, device=pts.device)
    if signal is not None:
        fl, val = signal
        cnt = ctypes.c_void_p(fl.value + 12) if signal_all else None
        w = wait.wait_args() if wait is not None else (None, 0, None, None, 0)
        _call("pcst_noise_mlp_ex", _ptr(pts), P, points_per_cloud, _ptr(cond), cond.shape[0],
              _ptr(blob), blob.numel(), _ptr(bias), precision, _ptr(out), fl, val, cnt, *w,
              _stream())
        return out
    if wait is not None and precision == 1 and P > 0:
        _call("pcst_noise_mlp_ex", _ptr(pts), P, points_per_cloud, _ptr(cond), cond.shape[0],
              _ptr(blob), blob.numel(), _ptr(bias), precision, _ptr(out), None, 0, None,
              *wait.wait_args(), _stream())
        return out
    _call("pcst_noise_mlp", _ptr(pts), P, points_per_cloud, _ptr(cond), cond.shape[0], _ptr(blob),
          blob.numel(), _ptr(bias), precision, _ptr(out), _stream())
    if wait is not None:
        wait.wait(torch.cuda.current_stream(pts.device))
    return out


# ----------------------------------------------------------------------------- CFG / DDIM update
def cfg_ddim_voxel_prep(x, eps, source, guidance_scale, coeffs, x_cat, vox_ws, copies=2, out=None,
                        pool_seed=None):
    """cfg_ddim_step(x, eps[:C], eps[C:], source, ...) of a CFG batch (x [C,N,3], eps [2C,N,3],
    x_cat [2C,N,3] receives the new x twice) fused with the first stage of the next
    voxel_downsample(new x, copies=copies, ws=vox_ws, prepped=True) (pcst.h).  pool_seed (the
    seed that downsample will take): also its pool-key histogram; it must then pass pool=True."""
    require_device(x, eps, source, x_cat, vox_ws)
    x, eps = _f32(x), _f32(eps)
    C, N, _ = x.shape
    if eps.shape != (2 * C, N, 3) or x_cat is None or x_cat.shape != (2 * C, N, 3):
        raise RuntimeError(f"cfg_ddim_voxel_prep: eps {tuple(eps.shape)} / x_cat must be {(2 * C, N, 3)}")
    if source is not None and source.shape != x.shape:
        raise RuntimeError("cfg_ddim_voxel_prep: source shape != x shape")
    need = ctypes.c_size_t(0)
    _call("pcst_voxel_copies_workspace_size", C, N, copies, ctypes.byref(need))
    if vox_ws.numel() < need.value:
        raise RuntimeError("cfg_ddim_voxel_prep: voxel workspace too small")
    if out is None:
        out = torch.empty_like(x)
    c1, c2, c3, c4 = (float(c) for c in coeffs)
    _call("pcst_cfg_ddim_voxel_prep", _ptr(x), _ptr(eps), _ptr(source), C, N, float(guidance_scale),
          c1, c2, c3, c4, _ptr(out), _ptr(x_cat), _ptr(vox_ws), copies,
          (pool_seed or 0) & (2**64 - 1), 0 if pool_seed is None else 1, _stream())
    return out


def cfg_ddim_step(x, eps_c, eps_u, source, guidance_scale, coeffs, x_cat=None, out=None):
    """coeffs = (sqrt(1-a_t), sqrt(a_t)+1e-8, sqrt(a_prev), sqrt(1-a_prev)) as fp32 values."""
    require_device(x, eps_c, eps_u, source, x_cat)
    x = _f32(x)
    if out is None:
        out = torch.empty_like(x)
    c1, c2, c3, c4 = (float(c) for c in coeffs)
    _call("pcst_cfg_ddim_step", _ptr(x), _ptr(eps_c), _ptr(eps_u), _ptr(source), x.numel(),
          float(guidance_scale), c1, c2, c3, c4, _ptr(out), _ptr(x_cat), _stream())
    return out


# ----------------------------------------------------------------------------- per-point linear
def pointwise_linear(X, W, scale=None, shift=None, relu=False, pool_ns=0):
    """X [M,K], W [O,K] -> act(scale*(X W^T)+shift) [M,O], or max-pooled [M/ns, O]."""
    require_device(X, W, scale, shift)
    X, W = _f32(X), _f32(W)
    M, K = X.shape
    O = W.shape[0]
    rows = M // pool_ns if pool_ns else M
    Y = torch.empty(rows, O, dtype=torch.float32, device=X.device)
    # converted operands stay bound to locals until the call returns (a temporary whose
    # block is freed before the launch could be handed to the next allocation)
    scale = None if scale is None else _f32(scale)
    shift = None if shift is None else _f32(shift)
    _call("pcst_pointwise_linear", _ptr(X), M, K, _ptr(W), O, _ptr(scale), _ptr(shift),
          int(relu), pool_ns, _ptr(Y), _stream())
    return Y


def relu_bwd(dy, y):
    """dy * [y > 0] in one pass (the ReLU backward of the per-point layers)."""
    require_device(dy, y)
    dy, y = _f32(dy), _f32(y)
    if dy.shape != y.shape:
        raise RuntimeError(f"relu_bwd: shape mismatch {tuple(dy.shape)} vs {tuple(y.shape)}")
    dz = torch.empty_like(dy)
    _call("pcst_relu_bwd", _ptr(dy), _ptr(y), dy.numel(), _ptr(dz), _stream())
    return dz


_HALVES = (torch.bfloat16, torch.float16)


def _f16_flag(half):
    """ABI format flag of a 16-bit dtype: 0 bfloat16, 1 float16 (pcst.h)."""
    if half not in _HALVES:
        raise RuntimeError(f"16-bit operand dtype must be bfloat16 or float16, got {half}")
    return 1 if half == torch.float16 else 0


def linear_wgrad(dZ, X, bias=True, bf16=False, half=torch.bfloat16):
    """dZ [M,O], X [M,I] -> (dW = dZ^T X [O,I], db = dZ^T 1 [O] or None); deterministic.
    bf16: operands rounded to the 16-bit `half` dtype (bfloat16 or float16) for the MFMA
    (autocast training), fp32 accumulation."""
    require_device(dZ, X)
    dZ, X = _f32(dZ), _f32(X)
    M, O = dZ.shape
    I = X.shape[1]
    if X.shape[0] != M:
        raise RuntimeError(f"linear_wgrad: row mismatch {tuple(dZ.shape)} vs {tuple(X.shape)}")
    fn = "pcst_linear_wgrad_bf16" if bf16 else "pcst_linear_wgrad"
    ws = _workspace(fn + "_workspace_size", M, I, O, device=dZ.device)
    dW = torch.empty(O, I, dtype=torch.float32, device=dZ.device)
    db = torch.empty(O, dtype=torch.float32, device=dZ.device) if bias else None
    if bf16:
        _call(fn, _ptr(dZ), _ptr(X), M, I, O, _ptr(dW), _ptr(db), _ptr(ws), _f16_flag(half),
              _stream())
    else:
        _call(fn, _ptr(dZ), _ptr(X), M, I, O, _ptr(dW), _ptr(db), _ptr(ws), _stream())
    return dW, db


def gemm_nt_bf16(A, B, scale=None, shift=None, relu=False, half=torch.bfloat16):
    """A [M,K], B [O,K] -> act(scale*(A B^T)+shift) [M,O] on 16-bit MFMA (operands rounded to
    `half`: bfloat16 or float16; fp32 accumulation)."""
    require_device(A, B, scale, shift)
    A, B = _f32(A), _f32(B)
    M, K = A.shape
    O = B.shape[0]
    if B.shape[1] != K:
        raise RuntimeError(f"gemm_nt_bf16: K mismatch {tuple(A.shape)} vs {tuple(B.shape)}")
    C = torch.empty(M, O, dtype=torch.float32, device=A.device)
    scale = None if scale is None else _f32(scale)
    shift = None if shift is None else _f32(shift)
    _call("pcst_gemm_nt_bf16", _ptr(A), M, K, _ptr(B), O, _ptr(scale), _ptr(shift),
          int(relu), _ptr(C), _f16_flag(half), _stream())
    return C


EP_F32, EP_BF16, EP_RESID_DROP, EP_RELU_MASK, EP_ADD, EP_COND, EP_RESID_DROP16, EP_ADD16 = range(8)
_EP_BF16_OUT = (EP_BF16, EP_RELU_MASK, EP_RESID_DROP16, EP_ADD16)
_EP_AUX16 = (EP_RELU_MASK, EP_RESID_DROP16, EP_ADD16)


def _f32_or_16(t, half):
    """(tensor, 16-bit flag): 16-bit tensors must be of the call's `half` dtype."""
    if t.dtype in _HALVES:
        if t.dtype != half:
            raise RuntimeError(f"16-bit operand is {t.dtype}, the call's format is {half}")
        return t.contiguous(), 1
    return _f32(t), 0


def _half_of(*ts, default=torch.bfloat16):
    """The 16-bit format of a call: that of its 16-bit tensors (all alike), else `default`."""
    hs = {t.dtype for t in ts if t is not None and t.dtype in _HALVES}
    if len(hs) > 1:
        raise RuntimeError(f"mixed 16-bit operand formats {hs}")
    return hs.pop() if hs else default


def resblock_fwd16(x, w1, b1, w2, b2, seed=0, p=0.0, mask_bits=False):
    """One residual block of the 16-bit residual stream in one launch (pcst_resblock_fwd16):
    x [M,256] 16-bit, w1 [512,256] / w2 [256,512] 16-bit (x's format), b1 [512] / b2 [256] fp32 ->
    (h [M,512] = relu(x w1^T + b1), x' [M,256] = x + Dropout_p(h w2^T + b2)), both 16-bit: the
    bits of gemm_ex EP_BF16 followed by EP_RESID_DROP16 under the same (seed, p).
    mask_bits=True: also the ReLU mask [h > 0] as int32 [M,16] bits (bit j of word w of row m =
    unit 32w + j), returned third, for resblock_bwd16(hbits=)."""
    require_device(x, w1, b1, w2, b2)
    half = x.dtype
    if half not in (torch.float16, torch.bfloat16):
        raise RuntimeError(f"resblock_fwd16: x must be float16 or bfloat16, got {x.dtype}")
    M = x.shape[0]
    if (x.dim() != 2 or x.shape[1] != 256 or tuple(w1.shape) != (512, 256)
            or tuple(w2.shape) != (256, 512) or w1.dtype != half or w2.dtype != half
            or b1.numel() != 512 or b2.numel() != 256):
        raise RuntimeError("resblock_fwd16: shapes are x [M,256], w1 [512,256], w2 [256,512], "
                           "b1 [512], b2 [256] in x's 16-bit format")
    x, w1, w2 = x.contiguous(), w1.contiguous(), w2.contiguous()
    h = torch.empty(M, 512, dtype=half, device=x.device)
    out = torch.empty(M, 256, dtype=half, device=x.device)
    hbits = torch.empty(M, 16, dtype=torch.int32, device=x.device) if mask_bits else None
    _call("pcst_resblock_fwd16", _ptr(x), M, _ptr(w1), _ptr(_f32(b1)), _ptr(w2), _ptr(_f32(b2)),
          int(seed) & (2**64 - 1), float(p), _ptr(h), _ptr(out), _ptr(hbits),
          1 if half == torch.float16 else 0, _stream())
    return (h, out, hbits) if mask_bits else (h, out)


def cast16_batch(tensors, half, transpose=None):
    """fp32 2-D tensors -> their 16-bit copies in `half` (float16 / bfloat16), each transposed where
    transpose[i], all in one launch (pcst_cast16_batch; the bits of t.to(half) / t.t().to(half))."""
    n = len(tensors)
    if n == 0:
        return []
    transpose = list(transpose) if transpose is not None else [False] * n
    if n > 64 or len(transpose) != n:
        raise RuntimeError("cast16_batch: at most 64 tensors, one transpose flag each")
    require_device(*tensors)
    src = [_f32(t.detach()) for t in tensors]
    if any(t.dim() != 2 for t in src):
        raise RuntimeError("cast16_batch: 2-D tensors only")
    sizes = [t.numel() for t in src]
    offs = np.cumsum([0] + [(z + 7) // 8 * 8 for z in sizes])  # 16-byte aligned slices
    flat = torch.empty(int(offs[-1]), dtype=half, device=src[0].device)
    outs = []
    for t, o, tr in zip(src, offs, transpose):
        r, c = t.shape
        outs.append(flat[int(o):int(o) + r * c].view(c, r) if tr else flat[int(o):int(o) + r * c].view(r, c))
    P = ctypes.c_void_p * n
    I32 = ctypes.c_int32 * n
    _call("pcst_cast16_batch", P(*[t.data_ptr() for t in src]), P(*[o.data_ptr() for o in outs]),
          I32(*[t.shape[0] for t in src]), I32(*[t.shape[1] for t in src]),
          I32(*[1 if tr else 0 for tr in transpose]), n, 1 if half == torch.float16 else 0, _stream())
    return outs


def resblock_bwd16(dd, w2t, w1t, h, g, seed=0, p=0.0, dropout_copy=False, hbits=None):
    """The backward products of one residual block in one launch (pcst_resblock_bwd16): dd, g
    [M,256] and h [M,512] 16-bit, w2t = W2^T [512,256] / w1t = W1^T [256,512] 16-bit ->
    (dz [M,512] = (dd W2) * [h > 0], g' [M,256] = g + dz W1, and with dropout_copy the previous
    block's dD' = g' keep / (1 - p) under (seed, p), else None), all 16-bit: the bits of gemm_ex
    EP_RELU_MASK (aux h) followed by EP_ADD16 (aux g, dropout_copy).  hbits: resblock_fwd16's
    mask bits [M,16], read instead of h (h may then be None)."""
    if h is None and hbits is None:
        raise RuntimeError("resblock_bwd16: give h or hbits")
    require_device(dd, w2t, w1t, g, *([h] if h is not None else []), *([hbits] if hbits is not None else []))
    half = dd.dtype
    if half not in (torch.float16, torch.bfloat16):
        raise RuntimeError(f"resblock_bwd16: dd must be float16 or bfloat16, got {dd.dtype}")
    M = dd.shape[0]
    if (dd.dim() != 2 or dd.shape[1] != 256 or tuple(w2t.shape) != (512, 256)
            or tuple(w1t.shape) != (256, 512) or (h is not None and tuple(h.shape) != (M, 512))
            or tuple(g.shape) != (M, 256)
            or (hbits is not None and (tuple(hbits.shape) != (M, 16) or hbits.dtype != torch.int32))
            or any(t.dtype != half for t in (w2t, w1t, g) + ((h,) if h is not None else ()))):
        raise RuntimeError("resblock_bwd16: shapes are dd [M,256], w2t [512,256], w1t [256,512], "
                           "h [M,512], g [M,256] in dd's 16-bit format")
    dd, w2t, w1t, g = (t.contiguous() for t in (dd, w2t, w1t, g))
    h = h.contiguous() if h is not None else None
    hbits = hbits.contiguous() if hbits is not None else None
    dz = torch.empty(M, 512, dtype=half, device=dd.device)
    g_out = torch.empty(M, 256, dtype=half, device=dd.device)
    dd_out = torch.empty(M, 256, dtype=half, device=dd.device) if dropout_copy else None
    _call("pcst_resblock_bwd16", _ptr(dd), M, _ptr(w2t), _ptr(w1t), _ptr(h), _ptr(g),
          int(seed) & (2**64 - 1), float(p), _ptr(dz), _ptr(g_out), _ptr(dd_out), _ptr(hbits),
          1 if half == torch.float16 else 0, _stream())
    return dz, g_out, dd_out


def gemm_ex(A, B, bias=None, relu=False, epilogue=EP_F32, aux=None, seed=0, p=0.0,
            group_rows=0, copy_bf16=False, half=None, dropout_copy=False, fp32_out=True):
    """A [M,K], B [O,K] (fp32 or 16-bit) -> epilogue(A B^T) on 16-bit MFMA (csrc/train_mlp.hip):
    EP_F32/EP_BF16 act(acc+bias) as fp32/16-bit, EP_RESID_DROP aux + dropout_p(acc+bias) (fp32),
    EP_RELU_MASK acc*[aux>0] (16-bit, aux 16-bit), EP_ADD acc + aux (fp32), EP_COND
    ((acc+bias) + aux[g,0]) + aux[g,1] with g = row // group_rows (fp32).  copy_bf16 (fp32
    outputs): also return a 16-bit copy, (C, C_16); with fp32_out=False (EP_COND) only C_16.
    EP_RESID_DROP16 / EP_ADD16: EP_RESID_DROP / EP_ADD with a 16-bit aux and output.
    dropout_copy (EP_BF16, EP_ADD16): also return half(C * keep / (1-p)) under (seed, p) --
    dropout_grad_bf16 of the stored C, fused -- as (C, dD).  `half` (bfloat16 or float16) is
    the 16-bit format; default: that of the 16-bit operands, else bfloat16."""
    require_device(A, B, bias, aux)
    half = half or _half_of(A, B, aux if epilogue in _EP_AUX16 else None)
    A, a16 = _f32_or_16(A, half)
    B, b16 = _f32_or_16(B, half)
    M, K = A.shape
    O = B.shape[0]
    if B.shape[1] != K:
        raise RuntimeError(f"gemm_ex: K mismatch {tuple(A.shape)} vs {tuple(B.shape)}")
    bias = None if bias is None else _f32(bias)
    if aux is not None:
        want = half if epilogue in _EP_AUX16 else torch.float32
        shape = (M // max(group_rows, 1), 2, O) if epilogue == EP_COND else (M, O)
        if aux.dtype != want or tuple(aux.shape) != shape:
            raise RuntimeError(f"gemm_ex: aux must be {want} {list(shape)}, got "
                               f"{aux.dtype} {list(aux.shape)}")
        aux = aux.contiguous()
    out_dtype = half if epilogue in _EP_BF16_OUT else torch.float32
    if not fp32_out and not (epilogue == EP_COND and copy_bf16):
        raise RuntimeError("gemm_ex: fp32_out=False is for EP_COND with copy_bf16")
    C = torch.empty(M, O, dtype=out_dtype, device=A.device) if fp32_out else None
    C2 = None
    if copy_bf16:
        if out_dtype != torch.float32:
            raise RuntimeError("gemm_ex: copy_bf16 needs an fp32 epilogue")
        C2 = torch.empty(M, O, dtype=half, device=A.device)
    if dropout_copy:
        if epilogue not in (EP_BF16, EP_ADD16) or copy_bf16:
            raise RuntimeError("gemm_ex: dropout_copy is for EP_BF16 / EP_ADD16")
        C2 = torch.empty(M, O, dtype=half, device=A.device)
    _call("pcst_gemm_ex", _ptr(A), a16, M, K, _ptr(B), b16, O, _ptr(bias), int(relu),
          int(epilogue), _ptr(aux), int(seed) & (2**64 - 1), float(p), int(group_rows), _ptr(C),
          _ptr(C2), _f16_flag(half), _stream())
    if not fp32_out:
        return C2
    return (C, C2) if copy_bf16 or dropout_copy else C


def dropout_grad_bf16(g, seed, p, half=torch.bfloat16):
    """Dropout backward with the mask regenerated from (seed, element index):
    half(g*keep/(1-p)), `half` bfloat16 or float16."""
    require_device(g)
    g = _f32(g)
    out = torch.empty(g.shape, dtype=half, device=g.device)
    _call("pcst_dropout_grad_bf16", _ptr(g), g.numel(), int(seed) & (2**64 - 1), float(p),
          _ptr(out), _f16_flag(half), _stream())
    return out


def linear_wgrad_ex(dZ, X, bias=True, half=None):
    """dZ [M,O], X [M,I] (fp32 or 16-bit) -> (dW = dZ^T X [O,I], db [O] or None) on 16-bit MFMA,
    deterministic; `half` as in gemm_ex."""
    require_device(dZ, X)
    half = half or _half_of(dZ, X)
    dZ, z16 = _f32_or_16(dZ, half)
    X, x16 = _f32_or_16(X, half)
    M, O = dZ.shape
    I = X.shape[1]
    if X.shape[0] != M:
        raise RuntimeError(f"linear_wgrad_ex: row mismatch {tuple(dZ.shape)} vs {tuple(X.shape)}")
    ws = _workspace("pcst_linear_wgrad_ex_workspace_size", M, I, O, device=dZ.device)
    dW = torch.empty(O, I, dtype=torch.float32, device=dZ.device)
    db = torch.empty(O, dtype=torch.float32, device=dZ.device) if bias else None
    _call("pcst_linear_wgrad_ex", _ptr(dZ), z16, _ptr(X), x16, M, I, O, _ptr(dW), _ptr(db),
          _ptr(ws), _f16_flag(half), _stream())
    return dW, db


def channel_stats(Z):
    """Per-channel (mean, biased var) of Z [M,O] as float64 device tensors (deterministic)."""
    require_device(Z)
    Z = _f32(Z)
    M, O = Z.shape
    ws = _workspace("pcst_channel_stats_workspace_size", O, device=Z.device)
    mean = torch.empty(O, dtype=torch.float64, device=Z.device)
    var = torch.empty(O, dtype=torch.float64, device=Z.device)
    _call("pcst_channel_stats", _ptr(Z), M, O, _ptr(mean), _ptr(var), _ptr(ws), _stream())
    return mean, var


def affine_act(Z, scale, shift, relu=True, pool_ns=0):
    require_device(Z, scale, shift)
    Z = _f32(Z)
    M, O = Z.shape
    rows = M // pool_ns if pool_ns else M
    Y = torch.empty(rows, O, dtype=torch.float32, device=Z.device)
    scale, shift = _f32(scale), _f32(shift)
    _call("pcst_affine_act", _ptr(Z), M, O, _ptr(scale), _ptr(shift), int(relu),
          pool_ns, _ptr(Y), _stream())
    return Y


# ----------------------------------------------------------------------------- SA training half
def bn_train_coeffs(mean, var, M, gamma, beta, eps, momentum, running_mean=None, running_var=None):
    """-> (scale fp32 [O], shift fp32 [O], invstd float64 [O]); running stats updated in place."""
    require_device(mean, var, gamma, beta)
    O = mean.shape[0]
    if mean.dtype != torch.float64 or var.dtype != torch.float64:
        raise RuntimeError("bn_train_coeffs: mean / var must be float64 (pcst_channel_stats)")
    gamma, beta = _f32(gamma), _f32(beta)
    for t in (running_mean, running_var):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise RuntimeError("bn_train_coeffs: running stats must be contiguous fp32")
    scale = torch.empty(O, dtype=torch.float32, device=mean.device)
    shift = torch.empty_like(scale)
    invstd = torch.empty(O, dtype=torch.float64, device=mean.device)
    _call("pcst_bn_train_coeffs", _ptr(mean), _ptr(var), int(M), O, _ptr(gamma), _ptr(beta),
          float(eps), float(momentum), _ptr(running_mean), _ptr(running_var), _ptr(scale),
          _ptr(shift), _ptr(invstd), _stream())
    return scale, shift, invstd


def bn_train_stats(Z, gamma, beta, eps, momentum, running_mean=None, running_var=None):
    """channel_stats then bn_train_coeffs in two launches (pcst_bn_train_stats, the same bits):
    -> (mean f64 [O], var f64 [O], scale f32 [O], shift f32 [O], invstd f64 [O]); running stats
    updated in place."""
    require_device(Z, gamma, beta)
    Z = _f32(Z)
    M, O = Z.shape
    gamma, beta = _f32(gamma), _f32(beta)
    for t in (running_mean, running_var):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise RuntimeError("bn_train_stats: running stats must be contiguous fp32")
    ws = _workspace("pcst_channel_stats_workspace_size", O, device=Z.device)
    dev = Z.device
    mean = torch.empty(O, dtype=torch.float64, device=dev)
    var = torch.empty(O, dtype=torch.float64, device=dev)
    scale = torch.empty(O, dtype=torch.float32, device=dev)
    shift = torch.empty_like(scale)
    invstd = torch.empty(O, dtype=torch.float64, device=dev)
    _call("pcst_bn_train_stats", _ptr(Z), M, O, _ptr(gamma), _ptr(beta), float(eps), float(momentum),
          _ptr(running_mean), _ptr(running_var), _ptr(mean), _ptr(var), _ptr(scale), _ptr(shift),
          _ptr(invstd), _ptr(ws), _stream())
    return mean, var, scale, shift, invstd


def bn_relu_maxpool(Z, scale, shift, ns):
    """-> (pooled [M/ns, O], arg int32 [M/ns, O]) of relu(scale*Z + shift)."""
    require_device(Z, scale, shift)
    Z, scale, shift = _f32(Z), _f32(scale), _f32(shift)
    M, O = Z.shape
    if M % ns:
        raise RuntimeError(f"bn_relu_maxpool: {M} rows not a multiple of {ns}")
    Y = torch.empty(M // ns, O, dtype=torch.float32, device=Z.device)
    arg = torch.empty(M // ns, O, dtype=torch.int32, device=Z.device)
    _call("pcst_bn_relu_maxpool", _ptr(Z), M, O, _ptr(scale), _ptr(shift), ns, _ptr(Y), _ptr(arg),
          _stream())
    return Y, arg


def bn_relu_bwd(Z, scale, shift, mean, invstd, gamma, dY=None, dP=None, arg=None, ns=0):
    """Backward of relu(BN_train(Z)) (+ max-pool when dP/arg given) -> (dZ, dgamma, dbeta)."""
    require_device(Z, scale, shift, mean, invstd, gamma, dY, dP, arg)
    Z, scale, shift, gamma = _f32(Z), _f32(scale), _f32(shift), _f32(gamma)
    M, O = Z.shape
    dY = None if dY is None else _f32(dY)
    dP = None if dP is None else _f32(dP)
    arg = None if arg is None else arg.contiguous()
    ws = _workspace("pcst_bn_relu_bwd_workspace_size", O, device=Z.device)
    dZ = torch.empty_like(Z)
    dgamma = torch.empty(O, dtype=torch.float32, device=Z.device)
    dbeta = torch.empty_like(dgamma)
    _call("pcst_bn_relu_bwd", _ptr(Z), M, O, _ptr(scale), _ptr(shift), _ptr(mean), _ptr(invstd),
          _ptr(gamma), _ptr(dY), _ptr(dP), _ptr(arg), int(ns), _ptr(dZ), _ptr(dgamma), _ptr(dbeta),
          _ptr(ws), _stream())
    return dZ, dgamma, dbeta


def group_gather_bwd(dgrouped, group_idx, N):
    """dgrouped [B,S,ns,3+C], group_idx [B,S,ns] -> dpoints [B,N,C] (deterministic)."""
    require_device(dgrouped, group_idx)
    dgrouped, group_idx = _f32(dgrouped), _i64(group_idx)
    B, S, ns, W = dgrouped.shape
    C = W - 3
    if tuple(group_idx.shape) != (B, S, ns):
        raise RuntimeError(f"group_gather_bwd: idx {tuple(group_idx.shape)} != {(B, S, ns)}")
    ws = _workspace("pcst_group_gather_bwd_workspace_size", B, S * ns, device=dgrouped.device)
    dP = torch.empty(B, N, C, dtype=torch.float32, device=dgrouped.device)
    _call("pcst_group_gather_bwd", _ptr(dgrouped), _ptr(group_idx), B, S, ns, N, C, _ptr(dP),
          _ptr(ws), _stream())
    return dP


def group_colsum16(g, B):
    """g [B*N, C] float16 / bfloat16 -> [B, C] float32: each cloud's column sums, rounded to g's
    16-bit type (the autocast reduction of a broadcast row; deterministic)."""
    require_device(g)
    if g.dtype not in (torch.float16, torch.bfloat16) or g.dim() != 2:
        raise RuntimeError(f"group_colsum16: need a 2-d float16/bfloat16 tensor, got {g.dtype} "
                           f"{tuple(g.shape)}")
    g = g.contiguous()
    M, C = g.shape
    if M % B:
        raise RuntimeError(f"group_colsum16: {M} rows do not split into {B} clouds")
    ws = _workspace("pcst_group_colsum16_workspace_size", B, C, device=g.device)
    out = torch.empty(B, C, dtype=torch.float32, device=g.device)
    _call("pcst_group_colsum16", _ptr(g), 1 if g.dtype == torch.float16 else 0, B, M // B, C,
          _ptr(out), _ptr(ws), _stream())
    return out


# ----------------------------------------------------------------------------- losses
def chamfer_fwd(pred, target, mode=0):
    """-> (chamfer [B], arg1 [B,N] int32, arg2 [B,M] int32).  mode: 0 auto (= 3), 1 exhaustive,
    2 grid-pruned, 3 hybrid (budgeted grid + exhaustive overflow rows); bit-identical results
    (pcst.h)."""
    require_device(pred, target)
    pred, target = _f32(pred), _f32(target)
    B, N, _ = pred.shape
    M = target.shape[1]
    dev = pred.device
    min1 = torch.empty(B, N, dtype=torch.float32, device=dev)
    min2 = torch.empty(B, M, dtype=torch.float32, device=dev)
    arg1 = torch.empty(B, N, dtype=torch.int32, device=dev)
    arg2 = torch.empty(B, M, dtype=torch.int32, device=dev)
    out = torch.empty(B, dtype=torch.float32, device=dev)
    ws = _workspace("pcst_chamfer_fwd_workspace_size", B, N, M, device=dev)
    _call("pcst_chamfer_fwd", _ptr(pred), _ptr(target), B, N, M, _ptr(min1), _ptr(arg1),
          _ptr(min2), _ptr(arg2), _ptr(out), int(mode), _ptr(ws), _stream())
    return out, arg1, arg2


def chamfer_bwd(pred, target, arg1, arg2, grad_out, need_pred=True, need_target=False):
    require_device(pred, target, arg1, arg2, grad_out)
    pred, target, grad_out = _f32(pred), _f32(target), _f32(grad_out)
    B, N, _ = pred.shape
    M = target.shape[1]
    ws = _workspace("pcst_chamfer_bwd_workspace_size", B, N, M, device=pred.device)
    gp = torch.zeros_like(pred) if need_pred else None
    gt = torch.zeros_like(target) if need_target else None
    arg1, arg2 = arg1.contiguous(), arg2.contiguous()
    _call("pcst_chamfer_bwd", _ptr(pred), _ptr(target), B, N, M, _ptr(arg1),
          _ptr(arg2), _ptr(grad_out), _ptr(gp), _ptr(gt), _ptr(ws), _stream())
    return gp, gt


def l1_fwd(a, b):
    require_device(a, b)
    a, b = _f32(a), _f32(b)
    ws = _workspace("pcst_l1_workspace_size", device=a.device)
    out = torch.empty((), dtype=torch.float32, device=a.device)
    _call("pcst_l1_fwd", _ptr(a), _ptr(b), a.numel(), _ptr(out), _ptr(ws), _stream())
    return out


def l1_bwd(a, b, grad_out):
    require_device(a, b, grad_out)
    a, b = _f32(a), _f32(b)
    ga = torch.empty_like(a)
    g = _f32(grad_out.reshape(1))
    _call("pcst_l1_bwd", _ptr(a), _ptr(b), a.numel(), _ptr(g), _ptr(ga), _stream())
    return ga


# ----------------------------------------------------------------------------- metrics
def knn_dist(P, Q, k=1, with_index=False):
    """P [B,N,3], Q [B,M,3] -> float64 distances [B,N,k] to the k nearest rows of Q (ascending,
    ties to the lower index) and, with_index, their int64 indices [B,N,k]."""
    require_device(P, Q)
    P, Q = _f32(P), _f32(Q)
    B, N, _ = P.shape
    M = Q.shape[1]
    if Q.shape[0] != B:
        raise RuntimeError(f"knn_dist: batch mismatch {tuple(P.shape)} vs {tuple(Q.shape)}")
    dist = torch.empty(B, N, k, dtype=torch.float64, device=P.device)
    idx = torch.empty(B, N, k, dtype=torch.int32, device=P.device) if with_index else None
    _call("pcst_knn_dist", _ptr(P), _ptr(Q), B, N, M, k, _ptr(dist), _ptr(idx), _stream())
    return (dist, idx.long()) if with_index else dist


def emd_greedy(P, Q):
    """Greedy-matching EMD of metrics.py:46-90 -> float32 [B]."""
    require_device(P, Q)
    P, Q = _f32(P), _f32(Q)
    B, N, _ = P.shape
    out = torch.empty(B, dtype=torch.float32, device=P.device)
    _call("pcst_emd_greedy", _ptr(P), _ptr(Q), B, N, Q.shape[1], _ptr(out), _stream())
    return out


# ----------------------------------------------------------------------------- offline preprocessing
def voxel_center_dist(points, xyz_min, voxel_size):
    """points [n,3] (device) -> (packed voxel key int64 [n], float64 distance to the voxel
    centre [n]) of preprocessing.py:71-85, with xyz_min / voxel_size computed by the caller."""
    require_device(points)
    points = _f32(points)
    n = points.shape[0]
    mn = (ctypes.c_float * 3)(*[float(v) for v in np.asarray(xyz_min, dtype=np.float32)])
    key = torch.empty(n, dtype=torch.int64, device=points.device)
    dist = torch.empty(n, dtype=torch.float64, device=points.device)
    ovf = torch.zeros(1, dtype=torch.int32, device=points.device)
    _call("pcst_voxel_center_dist", _ptr(points), n, ctypes.cast(mn, ctypes.c_void_p),
          ctypes.c_float(float(np.float32(voxel_size))), _ptr(key), _ptr(dist), _ptr(ovf), _stream())
    if int(ovf.item()):
        raise RuntimeError("pcst: voxel coordinates exceed 2^21 per axis")
    return key, dist


# ----------------------------------------------------------------------------- graph-replayable steps
def cfg_ddim_step_dcoef(x, eps_c, eps_u, source, guidance_scale, coef, x_cat=None, out=None):
    """cfg_ddim_step with the four fp32 coefficients read from the device tensor `coef` [4]."""
    require_device(x, eps_c, eps_u, source, x_cat, coef)
    if out is None:
        out = torch.empty_like(x)
    _call("pcst_cfg_ddim_step_dcoef", _ptr(x), _ptr(eps_c), _ptr(eps_u), _ptr(source), x.numel(),
          float(guidance_scale), _ptr(coef), _ptr(out), _ptr(x_cat), _stream())
    return out


def voxel_downsample_copies_dseed(points, target, seed_dev, copies):
    """voxel_downsample(points, target, copies=copies) with the subset seed read from the
    device tensor `seed_dev` (int64 [1], the same bits as the host seed)."""
    require_device(points, seed_dev)
    points = _f32(points)
    B, N, _ = points.shape
    dev = points.device
    ws = _workspace("pcst_voxel_copies_workspace_size", B, N, copies, device=dev)
    out_idx = torch.empty(copies * B, target, dtype=torch.int64, device=dev)
    out_pts = torch.empty(copies * B, target, 3, dtype=torch.float32, device=dev)
    _call("pcst_voxel_downsample_copies_dseed", _ptr(points), B, N, copies, target, _ptr(ws),
          _ptr(seed_dev), _ptr(out_idx), _ptr(out_pts), _stream())
    return out_pts, out_idx


# every public wrapper launches on its tensors' device (see _on_tensor_device)
_GUARDED = ("square_distance", "index_points", "fps", "ball_query", "group_gather",
            "voxel_downsample", "voxel_stats", "knn3_build", "knn3_query", "knn3_interp",
            "noise_cond", "noise_mlp", "cfg_ddim_step", "cfg_ddim_voxel_prep", "pointwise_linear", "relu_bwd",
            "linear_wgrad", "gemm_nt_bf16", "channel_stats", "bn_train_stats", "affine_act", "chamfer_fwd",
            "chamfer_bwd", "l1_fwd", "l1_bwd", "knn_dist", "emd_greedy", "voxel_center_dist",
            "cfg_ddim_step_dcoef", "voxel_downsample_copies_dseed", "bn_train_coeffs",
            "bn_relu_maxpool", "bn_relu_bwd", "group_gather_bwd", "group_colsum16", "resblock_fwd16", "resblock_bwd16", "cast16_batch",
            "gemm_ex", "dropout_grad_bf16",
            "linear_wgrad_ex", "knn_workspace", "voxel_copies_workspace", "knn3_rows_build",
            "knn3_rows_refs", "knn3_rows_query", "knn_rows_stats", "knn3_interp_rows")
for _name in _GUARDED:
    globals()[_name] = _on_tensor_device(globals()[_name])
del _name
