"""Loader for the native library `lib/libmipipe.so` (HIP kernels for gfx950 + C++ runtime).

`import torch` MUST happen before the library is loaded: torch ships its own HIP runtime and RCCL
(`libamdhip64.so.7`, `librccl.so.1`); loading ours afterwards makes the dynamic linker reuse those
exact objects (same SONAME), so kernels launched from C++ run on torch's streams/context and
device pointers are shared.  On a GPU box the library must load (no silent fallback): ops raise.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import threading

import torch  # noqa: F401  (see module docstring: must precede the dlopen)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
# MIPIPE_LIB selects another in-tree build of the library (A/B kernel experiments in one GPU call)
LIB_PATH = os.path.join(PKG_DIR, "lib", os.environ.get("MIPIPE_LIB", "libmipipe.so"))
BIN_DIR = os.path.join(PKG_DIR, "bin")

_lock = threading.Lock()
_lib = None

c_void_p, c_int, c_int64, c_float, c_double, c_char_p = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                                          ctypes.c_float, ctypes.c_double, ctypes.c_char_p)

_SIGS = {
    "mp_last_error": ([], c_char_p),
    "mp_version": ([], c_int),
    "mp_log_level": ([c_int], None),
    "mp_log_file": ([c_char_p], None),
    "mp_packed_bytes": ([c_int, c_int64, c_int64], c_int64),
    "mp_pack_type": ([c_int], c_int),
    "mp_pack_t16": ([c_int, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_int], c_int),
    "mp_dequant_row": ([c_int, c_void_p, c_void_p, c_int64], c_int),
    "mp_qdot_rows": ([c_int, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p], c_int),
    "mp_partition": ([c_void_p, c_int, c_double, c_double, c_void_p, c_int, c_int, c_void_p], c_int),
    "mp_gguf_open": ([c_char_p], c_void_p),
    "mp_gguf_close": ([c_void_p], None),
    "mp_gguf_json": ([c_void_p], c_char_p),
    "mp_model_config_json": ([c_char_p], c_char_p),
    "mp_op_gemv": ([c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p,
                    c_int, c_int, c_int, c_void_p], c_int),
    "mp_op_gemm": ([c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p,
                    c_int, c_int, c_void_p], c_int),
    "mp_op_gemm3": ([c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p,
                     c_int, c_int, c_int, c_void_p], c_int),
    "mp_set_gemm3_tuning": ([c_int, c_int, c_int, c_int], c_int),
    "mp_op_gemm4": ([c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p,
                     c_int, c_int, c_int, c_void_p], c_int),
    "mp_op_moe_route": ([c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p], c_int),
    "mp_op_moe_gemm4": ([c_int, c_int, c_void_p, ctypes.c_longlong, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                         c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p],
                        c_int),
    "mp_op_router_logits": ([c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p], c_int),
    "mp_op_gemm4_splitk": ([c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                            ctypes.c_longlong, c_void_p], c_int),
    "mp_op_quant_i8": ([c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p], c_int),
    "mp_op_gemm3_i8": ([c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int,
                        c_void_p, c_void_p, c_int, c_void_p], c_int),
    "mp_set_knob": ([c_char_p, c_int], c_int),
    "mp_reset_knob": ([c_char_p], c_int),
    "mp_op_unpack": ([c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p], c_int),
    "mp_op_rmsnorm": ([c_void_p, c_int, c_void_p, c_int, c_float, c_void_p, c_int, c_int, c_void_p], c_int),
    "mp_op_embed": ([c_int, c_void_p, c_int64, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p], c_int),
    "mp_op_rope_kv": ([c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                       c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "mp_op_attention": ([c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                         c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p], c_int),
    "mp_op_argmax": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "mp_op_attn_prefill": ([c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                            c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                            c_void_p], c_int),
    "mp_device_probe": ([c_int, c_void_p], c_int),
    "mp_op_gemv_fused": ([c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p,
                          c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_float, c_int, c_void_p, c_void_p,
                          c_void_p, c_int64, c_void_p], c_int),
    "mp_op_gemvs": ([c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
                     c_int, c_void_p, c_int, c_void_p, c_float, c_int, c_void_p, c_int, c_int, c_int, c_void_p], c_int),
    "mp_op_penalize": ([c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_float, c_float, c_float, c_void_p], c_int),
    "mp_op_hist_push": ([c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p], c_int),
    "mp_op_sample": ([c_void_p, c_int, c_int, c_int, c_float, c_int, c_float, c_float, ctypes.c_uint64, c_void_p,
                      c_void_p, c_void_p], c_int),
    "mp_tok_open": ([c_char_p], c_void_p),
    "mp_tok_close": ([c_void_p], None),
    "mp_tok_encode": ([c_void_p, c_char_p, c_int, c_int, c_void_p, c_int], c_int),
    "mp_tok_piece": ([c_void_p, c_int, c_void_p, c_int], c_int),
    "mp_tok_decode": ([c_void_p, c_void_p, c_int, c_void_p, c_int], c_int),
    "mp_tok_info": ([c_void_p, c_void_p], c_int),
    "mp_engine_create": ([c_char_p], c_void_p),
    "mp_engine_destroy": ([c_void_p], None),
    "mp_engine_info": ([c_void_p], c_char_p),
    "mp_engine_health": ([c_void_p], c_char_p),
    "mp_engine_save_state": ([c_void_p, c_char_p], c_char_p),
    "mp_plan_partition": ([c_char_p], c_char_p),
    "mp_engine_load_state": ([c_void_p, c_char_p], c_char_p),
    "mp_engine_trace": ([c_void_p, c_int, c_char_p], c_int),
    "mp_engine_generate": ([c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p], c_char_p),
    "mp_engine_spec_generate": ([c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p], c_char_p),
    "mp_engine_bench": ([c_void_p, c_int, c_int, c_int], c_char_p),
    "mp_engine_start": ([c_void_p, c_void_p, c_void_p, c_int], c_int),
    "mp_engine_admit": ([c_void_p, c_void_p, c_void_p, c_void_p, c_int], c_int),
    "mp_engine_release": ([c_void_p, c_int], c_int),
    "mp_engine_decode": ([c_void_p, c_int], c_char_p),
    "mp_engine_tokens": ([c_void_p, c_void_p, c_int, c_int], c_int),
    "mp_engine_logits": ([c_void_p, c_int, c_void_p, c_int], c_int),
    "mp_rccl_unique_id": ([c_void_p], c_int),
    "mp_local_link_selftest": ([c_int, c_int, c_int64, c_int, c_int], c_int),
    "mp_rccl_selftest": ([c_int, c_void_p, c_int, c_int], c_char_p),
    "mp_rccl_loop_start": ([c_int, c_int64, c_int], c_int),
    "mp_rccl_loop_wait": ([], c_double),
    "mp_rccl_probe_devices": ([c_void_p, c_int], c_char_p),
    "mp_set_gemv_tpw": ([c_int], None),
    "mp_init_packed": ([c_void_p, ctypes.c_size_t, c_int, c_float, ctypes.c_uint64, c_void_p], c_int),
    "mp_tok_pretokenize": ([c_char_p, c_int], c_char_p),
}


def _lib_newer_than_sources() -> bool:
    lib_t = os.path.getmtime(LIB_PATH)
    for sub in ("csrc/kernels", "csrc/runtime"):
        d = os.path.join(REPO_DIR, sub)
        for f in os.listdir(d):
            if f.endswith((".hip", ".cpp", ".h", ".inc")) and os.path.getmtime(os.path.join(d, f)) > lib_t:
                return False
    return os.path.getmtime(os.path.join(REPO_DIR, "Makefile")) <= lib_t


def _make(*extra, quiet=True):
    cmd = ["make", "-C", REPO_DIR, "-j", str(min(16, os.cpu_count() or 4)), *extra]
    return subprocess.run(cmd, capture_output=quiet, text=True)


def build(force: bool = False, quiet: bool = True) -> str:
    """Compile the native library in-tree with hipcc (gfx950).

    Staleness is make's business (it tracks every kernel / runtime source and header): `make -q`
    tells whether the in-tree library is current, and an out-of-date one is rebuilt rather than
    tested against newer sources."""
    if not force and os.path.exists(LIB_PATH) and os.environ.get("MIPIPE_LIB"):
        return LIB_PATH   # an explicitly selected A/B build is used as is
    if not force and os.path.exists(LIB_PATH) and _lib_newer_than_sources():
        # the in-tree library is newer than every native source: current (also on a GPU box whose
        # snapshot carries the library but not the object files make would otherwise look for)
        return LIB_PATH
    if not force and os.path.exists(LIB_PATH):
        try:
            if _make("-q", "all", quiet=True).returncode == 0:
                return LIB_PATH
        except OSError:   # no make on this machine: use what is there
            return LIB_PATH
    r = _make(quiet=quiet)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + (r.stdout or "")[-4000:] + (r.stderr or "")[-4000:])
    return LIB_PATH


def lib():
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                build()
            L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (args, res) in _SIGS.items():
                fn = getattr(L, name, None)
                if fn is None:
                    continue
                fn.argtypes = args
                fn.restype = res
            _lib = L
        return _lib


def check(rc, what="native call"):
    if (isinstance(rc, int) and rc < 0) or rc is None:
        err = lib().mp_last_error()
        raise RuntimeError(f"{what} failed: {err.decode() if err else 'unknown error'}")
    return rc


def cstr(s: str) -> bytes:
    return s.encode("utf-8")


def jcall(fn, *args, what="native call"):
    r = fn(*args)
    if r is None:
        check(None, what)
    return json.loads(r.decode("utf-8"))
