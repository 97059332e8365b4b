"""ctypes binding of the host runtime (include/mmvae_host.h, lib/libmmvae_host.so).

MatrixMarket -> cell-major CSR loader (the reference's mtx_data_block_t, mmvae_io.hh:49-290),
the counter-based bootstrap index generator and the train_vae_model driver
(mmvae_alg.hh:200-333).  Raises MMVAEError when the library is missing.
"""
import ctypes
import os
import weakref

import numpy as np

from . import Engine, MMVAEError, lib as engine_lib

_HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "lib", "libmmvae_host.so"))
BIN_DIR = os.path.normpath(os.path.join(_HERE, "..", "..", "bin"))
HOST_HEADER_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "..", "include", "mmvae_host.h"))


class CSR(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int64), ("D", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("rowptr", ctypes.POINTER(ctypes.c_int64)), ("col", ctypes.POINTER(ctypes.c_int32)),
                ("val", ctypes.POINTER(ctypes.c_float))]


class TrainOpts(ctypes.Structure):
    _fields_ = [("batch_size", ctypes.c_int64), ("max_epoch", ctypes.c_int64), ("nboot", ctypes.c_int64),
                ("recording", ctypes.c_int64), ("kl_discount", ctypes.c_float), ("kl_max", ctypes.c_float),
                ("kl_min", ctypes.c_float), ("seed", ctypes.c_uint64), ("out", ctypes.c_char_p),
                ("verbose", ctypes.c_int32), ("rank", ctypes.c_int32), ("world", ctypes.c_int32)]


_hlib = None


def hlib():
    global _hlib
    if _hlib is not None:
        return _hlib
    if not os.path.exists(HOST_LIB_PATH):
        raise MMVAEError(f"host library not built: {HOST_LIB_PATH} (run __graft_entry__.build())")
    engine_lib()  # the host library links libmmvae.so
    L = ctypes.CDLL(HOST_LIB_PATH)
    i64, i32 = ctypes.c_int64, ctypes.c_int32
    sig = {
        "mmvae_mtx_read": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(CSR)]),
        "mmvae_csr_save": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(CSR)]),
        "mmvae_csr_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(CSR)]),
        "mmvae_csr_free": (None, [ctypes.POINTER(CSR)]),
        "mmvae_mtx_read_dense_t": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(i64),
                                                  ctypes.POINTER(i64), ctypes.POINTER(ctypes.POINTER(ctypes.c_float))]),
        "mmvae_free": (None, [ctypes.c_void_p]),
        "mmvae_mtx_write_ones": (ctypes.c_int, [ctypes.c_char_p, i64]),
        "mmvae_mtx_build_index": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p]),
        "mmvae_mtx_read_index": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(i64)),
                                                ctypes.POINTER(i64)]),
        "mmvae_mtx_write_csr": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(CSR)]),
        "mmvae_host_last_error": (ctypes.c_char_p, []),
        "mmvae_train_opts_default": (None, [ctypes.POINTER(TrainOpts)]),
        "mmvae_ridx": (i64, [ctypes.c_uint64, i64, i64, i64, i64, i64]),
        "mmvae_train": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TrainOpts), ctypes.POINTER(ctypes.c_float)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _hlib = L
    return L


def _err(what, rc):
    raise MMVAEError(f"{what} failed ({rc}): {hlib().mmvae_host_last_error().decode()}")


def _owned(ptr, n):
    """numpy view of a malloc'd C array of n elements that frees it (mmvae_free) when the last
    view is gone: the loader's buffers are handed over without a copy."""
    a = np.ctypeslib.as_array(ptr, shape=(max(n, 1),))
    weakref.finalize(a, hlib().mmvae_free, ctypes.cast(ptr, ctypes.c_void_p))
    return a[:n]


def _take(c):
    rp = _owned(c.rowptr, c.N + 1)
    col = _owned(c.col, c.nnz)
    val = _owned(c.val, c.nnz)
    return rp, col, val, c.D


def mtx_read(path, threads=0):
    """MatrixMarket (plain/gzip/BGZF) -> (rowptr int64 [N+1], col int32, val f32, D)."""
    c = CSR()
    rc = hlib().mmvae_mtx_read(os.fsencode(path), threads, ctypes.byref(c))
    if rc:
        _err("mtx_read", rc)
    return _take(c)


def csr_save(path, rowptr, col, val, D):
    c, keep = _csr_struct(rowptr, col, val, D)
    rc = hlib().mmvae_csr_save(os.fsencode(path), ctypes.byref(c))
    if rc:
        _err("csr_save", rc)


def csr_load(path):
    c = CSR()
    rc = hlib().mmvae_csr_load(os.fsencode(path), ctypes.byref(c))
    if rc:
        _err("csr_load", rc)
    return _take(c)


def mtx_read_dense_t(path, threads=0):
    """Covariate MatrixMarket (rows = covariates, columns = cells) -> dense [N, C] f32."""
    N, C = ctypes.c_int64(), ctypes.c_int64()
    p = ctypes.POINTER(ctypes.c_float)()
    rc = hlib().mmvae_mtx_read_dense_t(os.fsencode(path), threads, ctypes.byref(N), ctypes.byref(C), ctypes.byref(p))
    if rc:
        _err("mtx_read_dense_t", rc)
    out = np.ctypeslib.as_array(p, shape=(N.value * C.value,)).copy().reshape(N.value, C.value)
    hlib().mmvae_free(p)
    return out


def mtx_write_ones(path, N):
    rc = hlib().mmvae_mtx_write_ones(os.fsencode(path), N)
    if rc:
        _err("mtx_write_ones", rc)


def _csr_struct(rowptr, col, val, D):
    rp = np.ascontiguousarray(rowptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    vl = np.ascontiguousarray(val, np.float32)
    c = CSR(rp.size - 1, D, cl.size, rp.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            cl.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), vl.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return c, (rp, cl, vl)


def mtx_write_csr(path, rowptr, col, val, D):
    """Cell-major CSR -> genes x cells BGZF MatrixMarket, sorted by cell."""
    c, keep = _csr_struct(rowptr, col, val, D)
    rc = hlib().mmvae_mtx_write_csr(os.fsencode(path), ctypes.byref(c))
    if rc:
        _err("mtx_write_csr", rc)


def mtx_build_index(mtx, index_file=None):
    """build_mmutil_index (mmutil_index.hh:138-190): ${mtx}.index as gzip 'col voff' text."""
    rc = hlib().mmvae_mtx_build_index(os.fsencode(mtx), os.fsencode(index_file) if index_file else None)
    if rc:
        _err("mtx_build_index", rc)
    return index_file or mtx + ".index"


def mtx_read_index(index_file):
    """read_mmutil_index (mmutil_index.hh:192-228): voff per column, gaps back-filled."""
    p = ctypes.POINTER(ctypes.c_int64)()
    n = ctypes.c_int64()
    rc = hlib().mmvae_mtx_read_index(os.fsencode(index_file), ctypes.byref(p), ctypes.byref(n))
    if rc:
        _err("mtx_read_index", rc)
    out = np.ctypeslib.as_array(p, shape=(n.value,)).copy()
    hlib().mmvae_free(p)
    return out


def ridx(seed, epoch, batch, boot, B):
    """Bootstrap indices of one resample (the counter-based stand-in for mmvae_alg.hh:292-293)."""
    f = hlib().mmvae_ridx
    return np.array([f(seed, epoch, batch, boot, j, B) for j in range(B)], dtype=np.int64)


def default_train_opts(**kw):
    o = TrainOpts()
    hlib().mmvae_train_opts_default(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v.encode() if isinstance(v, str) else v)
    return o


def train(engine: Engine, **kw):
    """mmvae_train on an engine with its dataset uploaded; returns the per-epoch scores."""
    o = default_train_opts(**kw)
    scores = np.zeros(max(o.max_epoch, 1), dtype=np.float32)
    rc = hlib().mmvae_train(engine._h, ctypes.byref(o), scores.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    if rc:
        _err("train", rc)
    return scores[:o.max_epoch]
