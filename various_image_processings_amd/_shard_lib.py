"""ctypes binding of include/vip_shard.h (libvip_shard.so: row-sharded frames with an
RCCL halo exchange). Loaded only by callers that shard, so that the filters alone never
load RCCL. No fallback: a missing library raises."""
from __future__ import annotations

import ctypes
import os
import threading

from . import _lib

LIB_PATH = os.path.join(_lib._HERE, "libvip_shard.so")

VIP_ERR_COMM = 10004
VIP_ERR_COMM_TIMEOUT = 10005
VIP_ERR_UNSUPPORTED = 10006
GRAPH_MIN_RCCL_VERSION = 22707  # vip_shard_set_graph needs RCCL >= 2.27.7
VIP_SHARD_ID_BYTES = 128
VIP_SHARD_RCCL = 0
VIP_SHARD_LOCAL = 1

_i, _p, _f, _s = ctypes.c_int, ctypes.c_void_p, ctypes.c_float, ctypes.c_size_t
_ip = ctypes.POINTER(ctypes.c_int)
_pp = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes); every entry point declared in include/vip_shard.h
SIGNATURES = {
    "vip_shard_rows": (_i, [_i, _i, _i, _ip, _ip]),
    "vip_shard_unique_id": (_i, [_p]),
    "vip_shard_create": (_i, [_pp, _i, _i, _i, _i, _f, _f, _i, _i, _i, _p, _i]),
    "vip_shard_create_texture": (_i, [_pp, _i, _i, _i, _i, _i, _i, _i, _p, _i]),
    "vip_shard_create_group": (_i, [_pp, _i, _i, _ip, _i, _i, _i, _i, _f, _f, _i, _i]),
    "vip_shard_create_group_texture": (_i, [_pp, _i, _i, _ip, _i, _i, _i, _i, _i, _i]),
    "vip_shard_geometry": (_i, [_p, _ip, _ip, _ip]),
    "vip_shard_set_split": (_i, [_p, _i]),
    "vip_shard_run": (_i, [_p, _p, _p, _s, _p]),
    "vip_shard_run_timed": (_i, [_p, _p, _p, _s, _p, _pp]),
    "vip_shard_run_batch": (_i, [_p, _i, _pp, _pp, _s, _p]),
    "vip_shard_run_group": (_i, [_pp, _i, _pp, _pp, _s, _pp]),
    "vip_shard_set_graph": (_i, [_p, _i]),
    "vip_shard_set_frames_launch": (_i, [_p, _i, _i]),
    "vip_shard_graph_count": (_i, [_p, _ip]),
    "vip_shard_rccl_version": (_i, [_ip]),
    "vip_shard_comm_info": (_i, [_p, _ip, _ip, _ip]),
    "vip_shard_pci_bus_id": (_i, [_p, ctypes.c_char_p, _i]),
    "vip_shard_create_loopback": (_i, [_pp, _i, _i, _i, _i, _f, _f, _i, _i, _i, _i, _i]),
    "vip_shard_last_error": (ctypes.c_char_p, []),
    "vip_shard_destroy": (_i, [_p]),
}

_lock = threading.Lock()
_lib_shard = None


class ShardError(_lib.VipError):
    def __init__(self, func: str, code: int):
        self.code = code
        if code in (VIP_ERR_COMM, VIP_ERR_COMM_TIMEOUT, VIP_ERR_UNSUPPORTED):
            detail = lib().vip_shard_last_error().decode(errors="replace")
            what = {VIP_ERR_COMM: "RCCL error", VIP_ERR_COMM_TIMEOUT: "timeout"}.get(code, "unsupported")
            RuntimeError.__init__(self, f"{func} failed with status {code}: {what}: {detail}")
        else:
            super().__init__(func, code)


def lib() -> ctypes.CDLL:
    global _lib_shard
    with _lock:
        if _lib_shard is None:
            _lib.lib()  # libvip_hip.so first (the shard library links it)
            if not os.path.exists(LIB_PATH):
                raise ImportError(f"{LIB_PATH} is not built; run __graft_entry__.build()")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib_shard = handle
    return _lib_shard


def call(name: str, *args) -> None:
    code = getattr(lib(), name)(*args)
    if code != 0:
        raise ShardError(name, code)
