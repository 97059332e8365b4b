"""CPU tests of the host runtime (libmmvae_host.so): the MatrixMarket loader against a numpy
parse of the same files (plain text, gzip, BGZF; shuffled entries, '%' lines in the body,
short lines, duplicates where the last entry wins as in mmvae_io.hh:115-123), the CSR cache,
the covariate reader, the all-ones covariate writer, the bootstrap index generator, every
symbol of include/mmvae_host.h, and the CLIs' argument handling (no GPU needed)."""
import ctypes
import gzip
import os
import re
import struct
import subprocess
import zlib

import numpy as np
import pytest

import mmvae_amd
from mmvae_amd import host
from oracle import synth


def bgzf_compress(data: bytes) -> bytes:
    """Independent BGZF writer (SAM spec 4.1) for the loader tests."""
    out = bytearray()
    for i in range(0, max(len(data), 1), 65280):
        blk = data[i:i + 65280]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        cdata = c.compress(blk) + c.flush()
        bsize = 18 + len(cdata) + 8 - 1
        out += struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
        out += cdata + struct.pack("<II", zlib.crc32(blk) & 0xffffffff, len(blk))
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return bytes(out)


def mtx_text(rowptr, col, val, D, order=None, extra=()):
    N = rowptr.size - 1
    cells = np.repeat(np.arange(N), np.diff(rowptr))
    trip = list(zip(col + 1, cells + 1, val))
    if order is not None:
        trip = [trip[i] for i in order]
    lines = ["%%MatrixMarket matrix coordinate integer general", "% a comment",
             f"{D} {N} {len(trip)}"]
    for k, (g, c, v) in enumerate(trip):
        lines.append(f"{g} {c} {v:g}")
        if k == len(trip) // 2:
            lines.extend(extra)
    return ("\n".join(lines) + "\n").encode()


@pytest.fixture(scope="module")
def data():
    rp, col, val = synth.synth_csr(300, 500, lib_size=300.0, seed=7)
    return rp, col, val, 500


def check(path, rp, col, val, D):
    r2, c2, v2, D2 = host.mtx_read(path, threads=4)
    assert D2 == D
    np.testing.assert_array_equal(r2, rp)
    np.testing.assert_array_equal(c2, col)
    np.testing.assert_array_equal(v2, val.astype(np.float32))


@pytest.mark.parametrize("fmt", ["plain", "gzip", "bgzf"])
def test_mtx_read_formats(tmp_path, data, fmt):
    rp, col, val, D = data
    t = mtx_text(rp, col, val, D)
    p = tmp_path / f"x.mtx{'' if fmt == 'plain' else '.gz'}"
    p.write_bytes(t if fmt == "plain" else gzip.compress(t) if fmt == "gzip" else bgzf_compress(t))
    check(str(p), rp, col, val, D)


@pytest.mark.parametrize("window", ["4096", "70001", "67108864"])
def test_mtx_read_streamed_windows(tmp_path, data, monkeypatch, window):
    """Column-sorted BGZF input streams window by window straight into the CSR (no whole-text
    buffer): small windows split BGZF blocks and lines at arbitrary points; a mid-file comment and
    short lines; genes shuffled and duplicated inside cells (sorted, last one kept)."""
    rp, col, val, D = data
    monkeypatch.setenv("MMVAE_MTX_WINDOW", window)
    t = mtx_text(rp, col, val, D, extra=["% mid comment", "7 9", ""])
    p = tmp_path / "w.mtx.gz"
    p.write_bytes(bgzf_compress(t))
    check(str(p), rp, col, val, D)
    # cells stay grouped, genes inside each cell reversed + one duplicate (the last must win)
    N = rp.size - 1
    lines = ["%%MatrixMarket matrix coordinate real general", f"{D} {N} 0"]
    for c in range(N):
        s0, s1 = rp[c], rp[c + 1]
        for j in range(s1 - 1, s0 - 1, -1):
            lines.append(f"{col[j] + 1} {c + 1} {val[j] + 100:g}")
        if s1 > s0:
            lines.append(f"{col[s0] + 1} {c + 1} 0.5")       # duplicate of the first gene, appended last
            lines.extend(f"{col[j] + 1} {c + 1} {val[j]:g}" for j in range(s0, s1) if j != s0)
    q = tmp_path / "u.mtx.gz"
    q.write_bytes(bgzf_compress(("\n".join(lines) + "\n").encode()))
    want_v = val.astype(np.float32).copy()
    want_v[rp[:-1][np.diff(rp) > 0]] = 0.5
    check(str(q), rp, col, want_v, D)


def test_mtx_read_shuffled_comments_short_lines(tmp_path, data):
    rp, col, val, D = data
    order = np.random.default_rng(0).permutation(rp[-1])
    t = mtx_text(rp, col, val, D, order=order, extra=["% mid comment", "7 9", ""])
    p = tmp_path / "s.mtx.gz"
    p.write_bytes(bgzf_compress(t))
    check(str(p), rp, col, val, D)


def test_mtx_read_duplicates_last_wins(tmp_path):
    t = b"%%MatrixMarket matrix coordinate real general\n4 3 6\n2 1 1.5\n1 1 2\n2 1 7.25\n4 3 1e2\n3 3 -1\n4 3 3\n"
    p = tmp_path / "d.mtx"
    p.write_bytes(t)
    rp, col, val, D = host.mtx_read(str(p))
    assert D == 4
    np.testing.assert_array_equal(rp, [0, 2, 2, 4])
    np.testing.assert_array_equal(col, [0, 1, 2, 3])
    np.testing.assert_array_equal(val, np.float32([2, 7.25, -1, 3]))


def test_mtx_read_errors(tmp_path):
    p = tmp_path / "bad.mtx"
    p.write_bytes(b"%%MatrixMarket matrix coordinate real general\n3 2 1\n4 1 1\n")
    with pytest.raises(mmvae_amd.MMVAEError, match="outside"):
        host.mtx_read(str(p))
    with pytest.raises(mmvae_amd.MMVAEError):
        host.mtx_read(str(tmp_path / "missing.mtx"))


def test_csr_cache_roundtrip(tmp_path, data):
    rp, col, val, D = data
    host.csr_save(str(tmp_path / "c.bin"), rp, col, val, D)
    r2, c2, v2, D2 = host.csr_load(str(tmp_path / "c.bin"))
    assert D2 == D
    np.testing.assert_array_equal(r2, rp)
    np.testing.assert_array_equal(c2, col)
    np.testing.assert_array_equal(v2, val)


def test_covariate_reader_and_ones_writer(tmp_path):
    rng = np.random.default_rng(3)
    C, N = 3, 17
    m = rng.integers(0, 3, (C, N)).astype(np.float32)
    lines = ["%%MatrixMarket matrix coordinate real general", f"{C} {N} {int((m != 0).sum())}"]
    lines += [f"{i + 1} {j + 1} {m[i, j]:g}" for j in range(N) for i in range(C) if m[i, j] != 0]
    p = tmp_path / "cov.mtx"
    p.write_text("\n".join(lines) + "\n")
    np.testing.assert_array_equal(host.mtx_read_dense_t(str(p)), m.T)
    q = tmp_path / "ones.mtx.gz"
    host.mtx_write_ones(str(q), N)
    raw = q.read_bytes()
    assert raw[:4] == b"\x1f\x8b\x08\x04" and raw[12:14] == b"BC"        # BGZF, io.hh:230-242
    txt = gzip.decompress(raw).decode().splitlines()
    assert txt[0] == "%%MatrixMarket matrix coordinate integer general" and txt[1] == f"1 {N} {N}"
    np.testing.assert_array_equal(host.mtx_read_dense_t(str(q)), np.ones((N, 1), np.float32))


def test_ridx_deterministic_uniform():
    a = host.ridx(5, 2, 3, 1, 4096)
    b = host.ridx(5, 2, 3, 1, 4096)
    c = host.ridx(5, 2, 3, 2, 4096)
    np.testing.assert_array_equal(a, b)
    assert (a != c).mean() > 0.99
    assert a.min() >= 0 and a.max() < 4096
    h = np.bincount(host.ridx(1, 0, 0, 0, 64 * 400) % 64, minlength=64)
    assert h.min() > 300 and h.max() < 500


def test_host_library_exports_every_declared_symbol():
    src = re.sub(r"/\*.*?\*/", "", open(host.HOST_HEADER_PATH).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(mmvae_[a-z0-9_]+)\s*\(", src)))
    L = ctypes.CDLL(host.HOST_LIB_PATH)
    assert len(names) >= 11
    assert not [n for n in names if not hasattr(L, n)]


@pytest.mark.parametrize("exe", ["nb_vae_main", "vmf_vae_main"])
def test_cli_arguments_without_gpu(tmp_path, exe):
    b = os.path.join(host.BIN_DIR, exe)
    r = subprocess.run([b, "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--mtx" in r.stderr
    r = subprocess.run([b, "--mtx", str(tmp_path / "nope.mtx"), "--out", str(tmp_path / "o")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "missing mtx" in r.stderr
    p = tmp_path / "x.mtx"
    p.write_text("%%MatrixMarket matrix coordinate integer general\n3 2 2\n1 1 4\n3 2 1\n")
    r = subprocess.run([b, "--mtx", str(p), "--out", str(tmp_path / "o"), "--mean_encoding" if exe == "nb_vae_main"
                        else "--encoding", ",".join(["100"] * 17)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "at most 16 hidden" in r.stderr  # checked before any device
    r = subprocess.run([b, "--mtx", str(p), "--out", str(tmp_path / "o"), "--dtype", "bf61"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "unknown --dtype bf61" in r.stderr and "fp8" in r.stderr


# ---- ${mtx}.index (mmutil_index.hh:38-228) ----------------------------------------------------
def _bgzf_blocks(raw):
    """(file offset, uncompressed start, uncompressed length) of every BGZF member."""
    out, p, u = [], 0, 0
    while p < len(raw):
        xlen = struct.unpack_from("<H", raw, p + 10)[0]
        bsize = struct.unpack_from("<H", raw, p + 16)[0]
        isize = struct.unpack_from("<I", raw, p + bsize + 1 - 4)[0]
        out.append((p, u, isize))
        p += bsize + 1
        u += isize
    return out


def _index_restated(raw):
    """mm_column_indexer_t restated: bgzf_tell after each line (bgzf.c:626-665: a line ending at
    a block's end leaves the reader at the next block, offset 0)."""
    blocks = [b for b in _bgzf_blocks(raw) if b[2] > 0]
    text = gzip.decompress(raw)

    def tell(u):
        for fo, us, ln in blocks:
            if us <= u < us + ln:
                return (fo << 16) | (u - us)
        return None

    pos, last_off, header, first_off, lineno, last_col, out = 0, 0, False, 0, 0, 0, []
    for line in text.split(b"\n")[:-1]:
        start_off = last_off
        pos += len(line) + 1
        last_off = tell(pos)
        if not line or line.startswith(b"%"):
            continue
        f = line.split()
        if not header:
            header, first_off = True, last_off
            continue
        col = int(f[1]) - 1
        if lineno == 0:
            last_col = col
            out.append((col, first_off))
        if col != last_col:
            out.append((col, start_off))
            last_col = col
        lineno += 1
    return out


def _line_at(raw, voff):
    """Seek a BGZF virtual offset and return the line found there (bgzf_seek + getline)."""
    addr, off = voff >> 16, voff & 0xffff
    data = b""
    for fo, us, ln in _bgzf_blocks(raw):
        if fo >= addr:
            data += zlib.decompressobj(16 + 15).decompress(raw[fo:])
            if b"\n" in data[off:]:
                break
    return data[off:].split(b"\n", 1)[0]


@pytest.mark.parametrize("window", [None, "4096", "70000"])
def test_index_builder_matches_restatement_and_seeks(tmp_path, data, monkeypatch, window):
    """The index is streamed window by window (MMVAE_MTX_WINDOW: a few BGZF blocks per window, so
    lines and block boundaries straddle windows); every window size gives the restated index."""
    if window:
        monkeypatch.setenv("MMVAE_MTX_WINDOW", window)
    rp, col, val, D = data
    raw = bgzf_compress(mtx_text(rp, col, val, D))  # ~ a few BGZF blocks, column-sorted
    p = tmp_path / "x.mtx.gz"
    p.write_bytes(raw)
    idx = host.mtx_build_index(str(p))
    assert idx == str(p) + ".index"
    pairs = [tuple(map(int, ln.split())) for ln in gzip.decompress(open(idx, "rb").read()).decode().splitlines()]
    assert pairs == _index_restated(raw)
    assert len(_bgzf_blocks(raw)) > 2
    voff = host.mtx_read_index(idx)
    N = rp.size - 1
    assert voff.size == N
    for j in range(N):
        if rp[j + 1] == rp[j]:
            continue
        line = _line_at(raw, int(voff[j])).split()
        assert int(line[1]) == j + 1 and int(line[0]) == col[rp[j]] + 1, (j, line)


def test_index_of_engine_writer_and_ones_file(tmp_path, data):
    rp, col, val, D = data
    p = str(tmp_path / "w.mtx.gz")
    host.mtx_write_csr(p, rp, col, val, D)
    r2, c2, v2, D2 = host.mtx_read(p)
    np.testing.assert_array_equal(r2, rp)
    np.testing.assert_array_equal(c2, col)
    raw = open(p, "rb").read()
    host.mtx_build_index(p, p + ".idx")
    pairs = [tuple(map(int, ln.split())) for ln in gzip.decompress(open(p + ".idx", "rb").read()).decode().splitlines()]
    assert pairs == _index_restated(raw)
    # the auto covariate file and its index (nb_vae_main.cc:68-73)
    ones = str(tmp_path / "o.covar.mtx.gz")
    host.mtx_write_ones(ones, 200000)
    os.environ["MMVAE_MTX_WINDOW"] = "100000"  # several windows over the ones file
    try:
        host.mtx_build_index(ones)
    finally:
        del os.environ["MMVAE_MTX_WINDOW"]
    v = host.mtx_read_index(ones + ".index")
    raw1 = open(ones, "rb").read()
    assert v.size == 200000 and len(_bgzf_blocks(raw1)) > 3
    for j in (0, 1, 4567, 99999, 199999):
        assert _line_at(raw1, int(v[j])) == f"1 {j + 1} 1".encode()


def test_index_builder_errors(tmp_path, data):
    rp, col, val, D = data
    plain = tmp_path / "p.mtx.gz"
    plain.write_bytes(gzip.compress(mtx_text(rp, col, val, D)))
    with pytest.raises(mmvae_amd.MMVAEError, match="not bgzipped"):
        host.mtx_build_index(str(plain))
    shuf = tmp_path / "s.mtx.gz"
    nnz = col.size
    shuf.write_bytes(bgzf_compress(mtx_text(rp, col, val, D, order=np.random.default_rng(0).permutation(nnz))))
    with pytest.raises(mmvae_amd.MMVAEError, match="sorted by columns"):
        host.mtx_build_index(str(shuf))
    # the last column empty: the reference refuses (mmutil_index.hh:171-179)
    rp2 = rp.copy()
    rp2[-1] = rp2[-2]
    short = tmp_path / "e.mtx.gz"
    short.write_bytes(bgzf_compress(mtx_text(rp2, col[:rp2[-1]], val[:rp2[-1]], D)))
    with pytest.raises(mmvae_amd.MMVAEError, match="Failed to index all the columns"):
        host.mtx_build_index(str(short))
