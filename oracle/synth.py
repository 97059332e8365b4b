"""Seeded synthetic single-cell count matrices (test infrastructure).

Distribution: gene propensity p_g ~ Gamma(0.3, 1) normalised over genes;
library size L_c ~ LogNormal(ln L0, 0.5); x_gc ~ Poisson(L_c * p_g * Gamma(2, 1/2)) (an NB
with r=2).  Returned as a cell-major CSR (rows = cells = MatrixMarket columns) with sorted
int32 gene indices and float32 values — the HBM layout of the engine.
"""
import numpy as np


def synth_csr(n_cells, n_genes, lib_size=2000.0, seed=0):
    rng = np.random.default_rng(seed)
    pg = rng.gamma(0.3, 1.0, size=n_genes)
    pg = pg / pg.sum()
    L = np.exp(np.log(lib_size) + 0.5 * rng.standard_normal(n_cells))
    rowptr = np.zeros(n_cells + 1, dtype=np.int64)
    cols, vals = [], []
    for c in range(n_cells):
        lam = L[c] * pg * rng.gamma(2.0, 0.5, size=n_genes)
        x = rng.poisson(lam)
        nz = np.nonzero(x)[0]
        cols.append(nz.astype(np.int32))
        vals.append(x[nz].astype(np.float32))
        rowptr[c + 1] = rowptr[c] + nz.size
    col = np.concatenate(cols) if cols else np.zeros(0, np.int32)
    val = np.concatenate(vals) if vals else np.zeros(0, np.float32)
    return rowptr, col, val


def densify(rowptr, col, val, rows, n_genes):
    """Dense [len(rows), D] float32 of the requested cell rows (duplicates allowed) —
    what ``mtx_data_block_t::read`` builds (reference mmvae_io.hh:208-245,122-131)."""
    out = np.zeros((len(rows), n_genes), dtype=np.float32)
    for j, r in enumerate(rows):
        a, b = rowptr[r], rowptr[r + 1]
        out[j, col[a:b]] = val[a:b]
    return out
