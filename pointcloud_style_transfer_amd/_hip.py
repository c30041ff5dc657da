"""ctypes binding of libpcst_hip.so (the C ABI declared in include/pcst.h).

This is the only place Python touches the native library.  Every wrapper takes
torch tensors that must live on the HIP device, passes raw device pointers,
shapes and torch's current stream, and raises RuntimeError with
pcst_last_error() on failure.  There is no CPU fallback: a missing library or a
CPU tensor is an error.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
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
}
_RESTYPES = {"pcst_version": ctypes.c_char_p, "pcst_last_error": ctypes.c_char_p}

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
            fn = getattr(L, name)
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
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


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
