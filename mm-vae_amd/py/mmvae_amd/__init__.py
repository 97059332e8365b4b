"""mmvae_amd — Python binding of the MI355X mmvae engine (ctypes over include/mmvae_capi.h).

Mirrors the reference's training interface: an :class:`Engine` holds one model
(``nbvae_t``, reference include/models/nb.hh:212-287) plus its Adam state and an
HBM-resident dataset; :meth:`Engine.step` is one ELBO step of ``train_vae_model``
(include/mmvae_alg.hh:300-310) and :meth:`Engine.eval_loss` the per-batch reported loss
(mmvae_alg.hh:277-285).  There is no CPU fallback: if ``lib/libmmvae.so`` is missing or no
GPU is present, constructing an Engine raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "lib", "libmmvae.so"))
if os.environ.get("MMVAE_LIB"):  # diagnostics: an alternative in-tree build (tools/build_variant.sh)
    LIB_PATH = os.path.abspath(os.environ["MMVAE_LIB"])
HEADER_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "..", "include", "mmvae_capi.h"))

MODEL_NB, MODEL_VMF = 0, 1
DTYPE_F32, DTYPE_BF16, DTYPE_BF16X3, DTYPE_FP8 = 0, 1, 2, 3
_DTYPES = {"f32": DTYPE_F32, "fp32": DTYPE_F32, "float32": DTYPE_F32, "bf16": DTYPE_BF16,
           "bf16x3": DTYPE_BF16X3, "x3": DTYPE_BF16X3, "fp8": DTYPE_FP8, "e4m3": DTYPE_FP8}


class MMVAEError(RuntimeError):
    pass


MAX_HIDDEN = 16  # MMVAE_MAX_HIDDEN (include/mmvae_capi.h)


class Cfg(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int32), ("dtype", ctypes.c_int32), ("D", ctypes.c_int64),
                ("C", ctypes.c_int64), ("K", ctypes.c_int64), ("H", ctypes.c_int64), ("R", ctypes.c_int64),
                ("max_batch", ctypes.c_int64), ("lr", ctypes.c_float), ("weight_decay", ctypes.c_float),
                ("grad_clip", ctypes.c_float), ("kappa_min", ctypes.c_float), ("kappa_max", ctypes.c_float),
                ("seed", ctypes.c_uint64), ("relu", ctypes.c_int32), ("n_enc_hidden", ctypes.c_int32),
                ("n_dec_hidden", ctypes.c_int32), ("enc_hidden", ctypes.c_int32 * MAX_HIDDEN),
                ("dec_hidden", ctypes.c_int32 * MAX_HIDDEN)]


class StepArgs(ctypes.Structure):
    _fields_ = [("cell_ids", ctypes.POINTER(ctypes.c_int64)), ("ridx", ctypes.POINTER(ctypes.c_int64)),
                ("B", ctypes.c_int64), ("n_total", ctypes.c_int64), ("row_offset", ctypes.c_int64),
                ("beta", ctypes.c_float), ("eps", ctypes.POINTER(ctypes.c_float)), ("step_id", ctypes.c_uint64),
                ("update", ctypes.c_int32)]


_lib = None


def lib():
    """Load libmmvae.so (built in-tree by ``make -C mm-vae_amd``); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MMVAEError(f"HIP library not built: {LIB_PATH} (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    h = ctypes.c_void_p
    i64, i32, f32p, i64p = ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int64)
    sig = {
        "mmvae_cfg_default": (None, [ctypes.POINTER(Cfg), i32]),
        "mmvae_create": (ctypes.c_int, [ctypes.POINTER(Cfg), ctypes.c_int, ctypes.POINTER(h)]),
        "mmvae_destroy": (ctypes.c_int, [h]),
        "mmvae_last_error": (ctypes.c_char_p, [h]),
        "mmvae_upload_csr": (ctypes.c_int, [h, i64p, ctypes.POINTER(ctypes.c_int32), f32p, i64, i64, f32p]),
        "mmvae_synth_csr": (ctypes.c_int, [h, i64, ctypes.c_double, ctypes.c_uint64, i64p]),
        "mmvae_stream_csr": (ctypes.c_int, [h, i64p, ctypes.POINTER(ctypes.c_int32), f32p, i64, i64, f32p]),
        "mmvae_dataset_size": (ctypes.c_int, [h, i64p, i64p]),
        "mmvae_param_shape": (ctypes.c_int, [h, i32, ctypes.POINTER(i32), i64p]),
        "mmvae_comm_allreduce": (ctypes.c_int, [h, f32p, i64]),
        "mmvae_get_rows": (ctypes.c_int, [h, i64p, i64, i64p, ctypes.POINTER(ctypes.c_int32), f32p, i64p]),
        "mmvae_num_params": (ctypes.c_int, [h, ctypes.POINTER(i32)]),
        "mmvae_param_info": (ctypes.c_int, [h, i32, ctypes.POINTER(ctypes.c_char_p), i64p, ctypes.POINTER(i32)]),
        "mmvae_set_param": (ctypes.c_int, [h, ctypes.c_char_p, f32p, i64]),
        "mmvae_get_param": (ctypes.c_int, [h, ctypes.c_char_p, f32p, i64]),
        "mmvae_get_grad": (ctypes.c_int, [h, ctypes.c_char_p, f32p, i64]),
        "mmvae_init_params": (ctypes.c_int, [h, ctypes.c_uint64]),
        "mmvae_reset_optimizer": (ctypes.c_int, [h]),
        "mmvae_run": (ctypes.c_int, [h, ctypes.POINTER(StepArgs), f32p, ctypes.POINTER(ctypes.c_double)]),
        "mmvae_step": (ctypes.c_int, [h, i64p, i64, i64p, ctypes.c_float, f32p, f32p]),
        "mmvae_eval": (ctypes.c_int, [h, i64p, i64, ctypes.c_float, f32p, f32p]),
        "mmvae_encode": (ctypes.c_int, [h, i64p, i64, f32p, f32p]),
        "mmvae_sync": (ctypes.c_int, [h]),
        "mmvae_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
        "mmvae_comm_init": (ctypes.c_int, [h, i32, i32, ctypes.c_void_p]),
        "mmvae_timing_enable": (ctypes.c_int, [h, i32]),
        "mmvae_timing_count": (ctypes.c_int, [h, ctypes.POINTER(i32)]),
        "mmvae_timing_get": (ctypes.c_int, [h, i32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double), i64p]),
        "mmvae_timing_reset": (ctypes.c_int, [h]),
        "mmvae_debug_copy": (ctypes.c_int, [h, i32, f32p, i64]),
        "mmvae_tiling_info": (ctypes.c_int, [h, ctypes.POINTER(i32)]),
        "mmvae_debug_poison": (ctypes.c_int, [h, i32]),
        "mmvae_graph_enable": (ctypes.c_int, [h, i32]),
        "mmvae_path": (ctypes.c_int, [h, ctypes.POINTER(ctypes.c_int32)]),
        "mmvae_graph_stats": (ctypes.c_int, [h, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
        "mmvae_lbessel": (ctypes.c_float, [ctypes.c_float, ctypes.c_float]),
        "mmvae_lbessel_grad": (ctypes.c_float, [ctypes.c_float, ctypes.c_float]),
        "mmvae_fasterlog": (ctypes.c_float, [ctypes.c_float]),
        "mmvae_fasterlgamma": (ctypes.c_float, [ctypes.c_float]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def default_cfg(model=MODEL_NB):
    c = Cfg()
    lib().mmvae_cfg_default(ctypes.byref(c), model)
    return c


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


class Engine:
    """One model + optimiser + HBM dataset on one GPU (the C handle)."""

    def __init__(self, D, K, C=1, H=1, R=1, max_batch=100, dtype="f32", model=MODEL_NB, device=0, seed=42,
                 lr=1e-3, kappa_min=0.1, kappa_max=10.0, relu=False, enc_hidden=(), dec_hidden=()):
        L = lib()
        c = default_cfg(model)
        c.D, c.K, c.C, c.H, c.R, c.max_batch = D, K, C, H, R, max_batch
        c.relu = 1 if relu else 0
        if len(enc_hidden) > MAX_HIDDEN or len(dec_hidden) > MAX_HIDDEN:
            raise MMVAEError(f"at most {MAX_HIDDEN} hidden encoder / decoder layers")
        c.n_enc_hidden, c.n_dec_hidden = len(enc_hidden), len(dec_hidden)
        for i, v in enumerate(enc_hidden):
            c.enc_hidden[i] = int(v)
        for i, v in enumerate(dec_hidden):
            c.dec_hidden[i] = int(v)
        c.dtype = _DTYPES[dtype] if isinstance(dtype, str) else int(dtype)
        c.seed, c.lr, c.kappa_min, c.kappa_max = seed, lr, kappa_min, kappa_max
        self.cfg = c
        self.D, self.K, self.C, self.H, self.R = D, K, C, H, R
        self.max_batch = max_batch
        self._h = ctypes.c_void_p()
        rc = L.mmvae_create(ctypes.byref(c), device, ctypes.byref(self._h))
        if rc != 0:
            raise MMVAEError(f"mmvae_create failed ({rc}): {L.mmvae_last_error(None).decode()}")
        self._step = 0

    # ---- plumbing ----
    def _chk(self, rc, what):
        if rc != 0:
            raise MMVAEError(f"{what} failed ({rc}): {lib().mmvae_last_error(self._h).decode()}")

    def close(self):
        if self._h:
            lib().mmvae_destroy(self._h)
            self._h = ctypes.c_void_p()
        self._stream_keep = None  # (after destroy: the engine no longer reads them)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- dataset ----
    def upload_csr(self, rowptr, col, val, covar=None):
        rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        val = _f32(val)
        N = rowptr.size - 1
        cv = _f32(covar) if covar is not None else None
        self._chk(lib().mmvae_upload_csr(self._h, _ptr(rowptr, ctypes.c_int64), _ptr(col, ctypes.c_int32),
                                         _ptr(val, ctypes.c_float), N, self.D,
                                         _ptr(cv, ctypes.c_float) if cv is not None else None), "upload_csr")
        self.N = N

    def stream_csr(self, rowptr, col, val, covar=None):
        """A host-resident dataset (mmvae_stream_csr): the arrays stay in host memory and every
        step gathers its batch's rows over PCIe; they are kept alive by the engine."""
        rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        val = _f32(val)
        cv = _f32(covar) if covar is not None else None
        N = rowptr.size - 1
        self._chk(lib().mmvae_stream_csr(self._h, _ptr(rowptr, ctypes.c_int64), _ptr(col, ctypes.c_int32),
                                         _ptr(val, ctypes.c_float), N, self.D,
                                         _ptr(cv, ctypes.c_float) if cv is not None else None), "stream_csr")
        self._stream_keep = (rowptr, col, val, cv)
        self.N = N

    def synth_csr(self, N, lib_size=2000.0, seed=0):
        nnz = ctypes.c_int64()
        self._chk(lib().mmvae_synth_csr(self._h, N, lib_size, seed, ctypes.byref(nnz)), "synth_csr")
        self.N = N
        return nnz.value

    def get_rows(self, rows):
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        rp = np.zeros(rows.size + 1, dtype=np.int64)
        nnz = ctypes.c_int64(0)
        self._chk(lib().mmvae_get_rows(self._h, _ptr(rows, ctypes.c_int64), rows.size, _ptr(rp, ctypes.c_int64),
                                       None, None, ctypes.byref(nnz)), "get_rows")
        col = np.zeros(max(nnz.value, 1), dtype=np.int32)
        val = np.zeros(max(nnz.value, 1), dtype=np.float32)
        self._chk(lib().mmvae_get_rows(self._h, _ptr(rows, ctypes.c_int64), rows.size, _ptr(rp, ctypes.c_int64),
                                       _ptr(col, ctypes.c_int32), _ptr(val, ctypes.c_float), ctypes.byref(nnz)),
                  "get_rows")
        return rp, col[:nnz.value], val[:nnz.value]

    # ---- parameters ----
    def param_info(self):
        n = ctypes.c_int32()
        self._chk(lib().mmvae_num_params(self._h, ctypes.byref(n)), "num_params")
        out = []
        for i in range(n.value):
            name, numel, reg = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int32()
            self._chk(lib().mmvae_param_info(self._h, i, ctypes.byref(name), ctypes.byref(numel), ctypes.byref(reg)),
                      "param_info")
            out.append((name.value.decode(), numel.value, bool(reg.value)))
        return out

    def set_param(self, name, arr):
        a = _f32(arr).ravel()
        self._chk(lib().mmvae_set_param(self._h, name.encode(), _ptr(a, ctypes.c_float), a.size), f"set_param {name}")

    def get_param(self, name, numel):
        a = np.zeros(numel, dtype=np.float32)
        self._chk(lib().mmvae_get_param(self._h, name.encode(), _ptr(a, ctypes.c_float), numel), f"get_param {name}")
        return a

    def get_grad(self, name, numel):
        a = np.zeros(numel, dtype=np.float32)
        self._chk(lib().mmvae_get_grad(self._h, name.encode(), _ptr(a, ctypes.c_float), numel), f"get_grad {name}")
        return a

    def set_params(self, d):
        for k, v in d.items():
            self.set_param(k, v)

    def params(self, registered_only=False):
        return {n: self.get_param(n, k) for n, k, r in self.param_info() if r or not registered_only}

    def grads(self):
        return {n: self.get_grad(n, k) for n, k, r in self.param_info() if r}

    def init_params(self, seed=0):
        self._chk(lib().mmvae_init_params(self._h, seed), "init_params")

    def reset_optimizer(self):
        self._chk(lib().mmvae_reset_optimizer(self._h), "reset_optimizer")

    # ---- steps ----
    def run(self, cell_ids, beta, eps=None, ridx=None, update=True, n_total=0, row_offset=0, step_id=None,
            sync=True):
        cells = np.ascontiguousarray(cell_ids, dtype=np.int64)
        a = StepArgs()
        a.cell_ids = _ptr(cells, ctypes.c_int64)
        rid = None
        if ridx is not None:
            rid = np.ascontiguousarray(ridx, dtype=np.int64)
            a.ridx = _ptr(rid, ctypes.c_int64)
        a.B = cells.size
        a.n_total = n_total
        a.row_offset = row_offset
        a.beta = beta
        ep = None
        if eps is not None:
            ep = _f32(eps).ravel()
            a.eps = _ptr(ep, ctypes.c_float)
        a.step_id = self._step if step_id is None else step_id
        a.update = 1 if update else 0
        if update:
            self._step += 1
        loss = ctypes.c_float()
        norm = ctypes.c_double()
        self._chk(lib().mmvae_run(self._h, ctypes.byref(a), ctypes.byref(loss) if sync else None,
                                  ctypes.byref(norm) if sync else None), "run")
        return (loss.value, norm.value) if sync else (None, None)

    def step(self, cell_ids, beta, eps=None, ridx=None, **kw):
        return self.run(cell_ids, beta, eps=eps, ridx=ridx, update=True, **kw)

    def eval_loss(self, cell_ids, beta, eps=None, **kw):
        return self.run(cell_ids, beta, eps=eps, update=False, **kw)[0]

    def encode(self, cell_ids):
        cells = np.ascontiguousarray(cell_ids, dtype=np.int64)
        m = np.zeros((cells.size, self.K), dtype=np.float32)
        lv = np.zeros((cells.size, self.K), dtype=np.float32)
        self._chk(lib().mmvae_encode(self._h, _ptr(cells, ctypes.c_int64), cells.size, _ptr(m, ctypes.c_float),
                                     _ptr(lv, ctypes.c_float)), "encode")
        return m, lv

    def sync(self):
        self._chk(lib().mmvae_sync(self._h), "sync")

    # ---- data parallel ----
    @staticmethod
    def comm_unique_id():
        buf = ctypes.create_string_buffer(128)
        rc = lib().mmvae_comm_unique_id(buf)
        if rc != 0:
            raise MMVAEError("comm_unique_id failed: " + lib().mmvae_last_error(None).decode())
        return bytes(buf.raw)

    def comm_init(self, rank, world, uid):
        """uid = the 128-byte RCCL id, or None for the local decomposition mode (no reduction)."""
        buf = ctypes.create_string_buffer(bytes(uid), 128) if uid is not None else None
        self._chk(lib().mmvae_comm_init(self._h, rank, world, buf), "comm_init")

    def tiling(self):
        """{'NT', 'split_enc', 'split_dec', 'split_ac', 'split_encb'} and tiles per split (tps_*)."""
        a = (ctypes.c_int32 * 5)()
        self._chk(lib().mmvae_tiling_info(self._h, a), "tiling_info")
        NT = a[0]
        out = {"NT": NT, "split_enc": a[1], "split_dec": a[2], "split_ac": a[3], "split_encb": a[4]}
        for k in ("enc", "dec", "ac", "encb"):
            out["tps_" + k] = -(-NT // out["split_" + k])
        return out

    def poison(self, byte):
        """Fill the per-step workspace with `byte` (test hook, mmvae_debug_poison)."""
        self._chk(lib().mmvae_debug_poison(self._h, int(byte)), "debug_poison")

    def path(self):
        """'fused' (the tile kernels) or 'wide' (dense batch + generic GEMMs: shapes beyond them)."""
        w = ctypes.c_int32()
        self._chk(lib().mmvae_path(self._h, ctypes.byref(w)), "path")
        return "wide" if w.value else "fused"

    def graph(self, on=True):
        """Capture / replay each step's device work as one hipGraph (mmvae_graph_enable)."""
        self._chk(lib().mmvae_graph_enable(self._h, 1 if on else 0), "graph_enable")

    def graph_stats(self):
        c, r = ctypes.c_int64(), ctypes.c_int64()
        self._chk(lib().mmvae_graph_stats(self._h, ctypes.byref(c), ctypes.byref(r)), "graph_stats")
        return {"captures": c.value, "replays": r.value}

    # ---- timing ----
    def timing(self, on=True):
        self._chk(lib().mmvae_timing_enable(self._h, 1 if on else 0), "timing_enable")

    def timing_reset(self):
        self._chk(lib().mmvae_timing_reset(self._h), "timing_reset")

    def timings(self):
        n = ctypes.c_int32()
        self._chk(lib().mmvae_timing_count(self._h, ctypes.byref(n)), "timing_count")
        out = {}
        for i in range(n.value):
            name, ms, cnt = ctypes.c_char_p(), ctypes.c_double(), ctypes.c_int64()
            self._chk(lib().mmvae_timing_get(self._h, i, ctypes.byref(name), ctypes.byref(ms), ctypes.byref(cnt)),
                      "timing_get")
            out[name.value.decode()] = (ms.value, cnt.value)
        return out


# ---- operators.hh scalars ----
def shard_batch(batch, B_global, N, rank, world):
    """Data-parallel batch selection (host logic, no GPU).

    The reference draws batch ``batch`` as the contiguous dataset rows (batch*B + j) % N,
    j < B (mmvae_alg.hh:264-266).  Under DP the global batch of B_global rows is split into
    ``world`` equal contiguous slices; rank r takes rows [r B/W, (r+1) B/W) of it.
    Returns (cell_ids int64 [B_global/world], row_offset = global index of the first row)."""
    if B_global % world:
        raise ValueError("global batch must divide evenly across ranks")
    b = B_global // world
    base = batch * B_global + rank * b
    return (base + np.arange(b, dtype=np.int64)) % N, rank * b


def lbessel(kappa, nu):
    return lib().mmvae_lbessel(kappa, nu)


def lbessel_grad(kappa, nu):
    return lib().mmvae_lbessel_grad(kappa, nu)


def fasterlog(x):
    return lib().mmvae_fasterlog(x)


def fasterlgamma(x):
    return lib().mmvae_fasterlgamma(x)
