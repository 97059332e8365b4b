// MatrixMarket (plain / gzip / BGZF) -> cell-major CSR, loaded once for an HBM-resident run.
//
// Replaces the reference's per-batch BGZF reader (mtx_data_block_t::read, mmvae_io.hh:208-245,
// over visit_bgzf_block, mmutil_bgzf_util.hh:53-151) with a one-time parallel load:
//   1. the compressed file is read whole; BGZF block boundaries come from each block's BSIZE
//      field, so blocks inflate independently on every worker (raw deflate, ISIZE-sized slots
//      of one text buffer); non-BGZF gzip streams inflate serially, plain text is used as is;
//   2. the text after the "rows cols nnz" header splits at line boundaries into one chunk per
//      worker; each parses its triplets (1-based; '%' lines and lines with < 3 fields skipped,
//      as mmutil_bgzf_util.hh:102-127 does);
//   3. per-chunk column histograms -> rowptr; entries scatter in file order; rows whose genes
//      are unsorted or repeated are sorted stably and deduplicated keeping the LAST entry (the
//      reference's dense scatter overwrites, mmvae_io.hh:115-123).
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cmath>
#include <unistd.h>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/mmvae_host.h"
#include "host_common.hh"

namespace mmvae_host {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int default_threads(int threads) {
    if (threads > 0) return threads;
    int n = (int)std::thread::hardware_concurrency();
    if (const char* e = std::getenv("OMP_NUM_THREADS")) {
        const int v = std::atoi(e);
        if (v > 0 && (n <= 0 || v < n)) n = v;
    }
    return std::max(1, std::min(n, 64));
}

template <class F>
void parallel_for(int nthreads, int64_t n, F&& f) {
    if (n <= 0) return;
    nthreads = (int)std::min<int64_t>(nthreads, n);
    if (nthreads <= 1) {
        f(0, (int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        const int64_t a = n * t / nthreads, b = n * (t + 1) / nthreads;
        th.emplace_back([&f, t, a, b] { f(t, a, b); });
    }
    for (auto& x : th) x.join();
}

static bool read_whole(const char* path, std::vector<unsigned char>& buf, std::string& err) {
    FILE* fp = std::fopen(path, "rb");
    if (!fp) {
        err = std::string("cannot open ") + path + ": " + std::strerror(errno);
        return false;
    }
    std::fseek(fp, 0, SEEK_END);
    const long sz = std::ftell(fp);
    std::fseek(fp, 0, SEEK_SET);
    if (sz < 0) {
        std::fclose(fp);
        err = std::string("cannot size ") + path;
        return false;
    }
    buf.resize((size_t)sz);
    size_t got = 0;
    while (got < buf.size()) {
        const size_t r = std::fread(buf.data() + got, 1, buf.size() - got, fp);
        if (r == 0) break;
        got += r;
    }
    std::fclose(fp);
    if (got != buf.size()) {
        err = std::string("short read on ") + path;
        return false;
    }
    return true;
}

struct BgzfBlock {
    size_t in_off, in_len, out_off, out_len;
    size_t file_off;  // the member's first byte (the block address of a BGZF virtual offset)
};

static uint32_t le32(const unsigned char* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Every gzip member carries a 'BC' extra subfield with BSIZE (SAM/BGZF spec): true -> blocks
static bool scan_bgzf(const std::vector<unsigned char>& b, std::vector<BgzfBlock>& blocks) {
    size_t p = 0, out = 0;
    while (p < b.size()) {
        if (p + 18 > b.size()) return false;
        if (b[p] != 31 || b[p + 1] != 139 || b[p + 2] != 8 || !(b[p + 3] & 4)) return false;
        const size_t xlen = b[p + 10] | (b[p + 11] << 8);
        size_t q = p + 12, qe = q + xlen;
        long bsize = -1;
        while (q + 4 <= qe && qe <= b.size()) {
            const int slen = b[q + 2] | (b[q + 3] << 8);
            if (b[q] == 'B' && b[q + 1] == 'C' && slen == 2 && q + 6 <= b.size()) bsize = b[q + 4] | (b[q + 5] << 8);
            q += 4 + (size_t)slen;
        }
        if (bsize < 0) return false;
        const size_t total = (size_t)bsize + 1, hdr = 12 + xlen;
        if (total < hdr + 8 || p + total > b.size()) return false;
        BgzfBlock blk;
        blk.file_off = p;
        blk.in_off = p + hdr;
        blk.in_len = total - hdr - 8;
        blk.out_len = le32(&b[p + total - 4]);
        blk.out_off = out;
        out += blk.out_len;
        blocks.push_back(blk);
        p += total;
    }
    return true;
}

// The whole BGZF blocks at the front of b[0, n): false if b does not start a BGZF block; the
// bytes of a trailing partial block are left (consumed = bytes of the whole blocks)
static bool scan_bgzf_window(const unsigned char* b, size_t n, std::vector<BgzfBlock>& blocks, size_t& consumed) {
    size_t p = 0, out = 0;
    blocks.clear();
    while (p + 18 <= n) {
        if (b[p] != 31 || b[p + 1] != 139 || b[p + 2] != 8 || !(b[p + 3] & 4)) return false;
        const size_t xlen = b[p + 10] | (b[p + 11] << 8);
        size_t q = p + 12;
        const size_t qe = q + xlen;
        if (qe > n) break;
        long bsize = -1;
        while (q + 4 <= qe) {
            const int slen = b[q + 2] | (b[q + 3] << 8);
            if (b[q] == 'B' && b[q + 1] == 'C' && slen == 2 && q + 6 <= n) bsize = b[q + 4] | (b[q + 5] << 8);
            q += 4 + (size_t)slen;
        }
        if (bsize < 0) return false;
        const size_t total = (size_t)bsize + 1, hdr = 12 + xlen;
        if (total < hdr + 8) return false;
        if (p + total > n) break;
        BgzfBlock blk;
        blk.file_off = p;
        blk.in_off = p + hdr;
        blk.in_len = total - hdr - 8;
        blk.out_len = le32(&b[p + total - 4]);
        blk.out_off = out;
        out += blk.out_len;
        blocks.push_back(blk);
        p += total;
    }
    consumed = p;
    return true;
}

static bool inflate_raw(const unsigned char* in, size_t in_len, char* out, size_t out_len) {
    z_stream s;
    std::memset(&s, 0, sizeof(s));
    if (inflateInit2(&s, -15) != Z_OK) return false;
    s.next_in = const_cast<unsigned char*>(in);
    s.avail_in = (uInt)in_len;
    s.next_out = reinterpret_cast<unsigned char*>(out);
    s.avail_out = (uInt)out_len;
    const int r = inflate(&s, Z_FINISH);
    const bool ok = (r == Z_STREAM_END) && s.total_out == out_len;
    inflateEnd(&s);
    return ok || (out_len == 0);
}

// serial inflate of (possibly multi-member) gzip
static bool inflate_gzip(const std::vector<unsigned char>& in, std::vector<char>& out, std::string& err) {
    z_stream s;
    std::memset(&s, 0, sizeof(s));
    if (inflateInit2(&s, 15 + 32) != Z_OK) {
        err = "inflateInit2 failed";
        return false;
    }
    s.next_in = const_cast<unsigned char*>(in.data());
    s.avail_in = (uInt)std::min<size_t>(in.size(), 1u << 30);
    size_t consumed_base = 0;
    out.resize(std::max<size_t>(in.size() * 4, 1 << 20));
    size_t produced = 0;
    for (;;) {
        if (produced == out.size()) out.resize(out.size() * 2);
        s.next_out = reinterpret_cast<unsigned char*>(out.data() + produced);
        s.avail_out = (uInt)std::min<size_t>(out.size() - produced, 1u << 30);
        const uInt before = s.avail_out;
        const int r = inflate(&s, Z_NO_FLUSH);
        produced += before - s.avail_out;
        const size_t consumed = consumed_base + (size_t)(s.next_in - (in.data() + consumed_base));
        if (r == Z_STREAM_END) {
            if (consumed >= in.size()) break;
            inflateReset(&s);  // next gzip member
        } else if (r != Z_OK && r != Z_BUF_ERROR) {
            inflateEnd(&s);
            err = "gzip stream is corrupt";
            return false;
        }
        if (s.avail_in == 0) {
            if (consumed >= in.size()) break;
            consumed_base = consumed;
            s.next_in = const_cast<unsigned char*>(in.data() + consumed);
            s.avail_in = (uInt)std::min<size_t>(in.size() - consumed, 1u << 30);
        }
    }
    inflateEnd(&s);
    out.resize(produced);
    return true;
}

bool load_text(const char* path, int threads, std::vector<char>& text, std::string& err) {
    std::vector<unsigned char> raw;
    if (!read_whole(path, raw, err)) return false;
    if (raw.size() >= 2 && raw[0] == 0x1f && raw[1] == 0x8b) {
        std::vector<BgzfBlock> blocks;
        if (scan_bgzf(raw, blocks)) {
            const size_t total = blocks.empty() ? 0 : blocks.back().out_off + blocks.back().out_len;
            text.resize(total);
            std::atomic<bool> ok{true};
            parallel_for(threads, (int64_t)blocks.size(), [&](int, int64_t a, int64_t bnd) {
                for (int64_t i = a; i < bnd; ++i) {
                    const BgzfBlock& k = blocks[(size_t)i];
                    if (!inflate_raw(raw.data() + k.in_off, k.in_len, text.data() + k.out_off, k.out_len)) ok = false;
                }
            });
            if (!ok) {
                err = std::string("corrupt BGZF block in ") + path;
                return false;
            }
            return true;
        }
        return inflate_gzip(raw, text, err);
    }
    text.assign(raw.begin(), raw.end());
    return true;
}

// ---- triplet parsing ------------------------------------------------------------------------
static inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

static inline float parse_float(const char* a, const char* e) {
    // fast path: optional sign + digits (integer counts); otherwise strtof on a copy
    const char* p = a;
    bool neg = false;
    if (p < e && (*p == '-' || *p == '+')) neg = (*p++ == '-');
    uint64_t v = 0;
    const char* d0 = p;
    while (p < e && *p >= '0' && *p <= '9' && p - d0 < 18) v = v * 10 + (uint64_t)(*p++ - '0');
    if (p == e && p > d0) return neg ? -(float)v : (float)v;
    char tmp[64];
    const size_t n = std::min<size_t>((size_t)(e - a), sizeof(tmp) - 1);
    std::memcpy(tmp, a, n);
    tmp[n] = 0;
    return std::strtof(tmp, nullptr);
}

static inline int64_t parse_int(const char* a, const char* e) {
    int64_t v = 0;
    const char* p = a;
    bool neg = false;
    if (p < e && (*p == '-' || *p == '+')) neg = (*p++ == '-');
    while (p < e && *p >= '0' && *p <= '9') v = v * 10 + (*p++ - '0');
    return neg ? -v : v;
}

struct Chunk {
    std::vector<int32_t> cell, gene;
    std::vector<float> val;
    int64_t cmin = INT64_MAX, cmax = -1;
    std::string err;
};

// visit each line of [p, e): f(tokens[3]) for lines with >= 3 fields, skipping '%' lines
static void parse_chunk(const char* p, const char* e, int64_t D, int64_t N, Chunk& ch) {
    ch.cell.reserve((size_t)((e - p) / 10));
    ch.gene.reserve((size_t)((e - p) / 10));
    ch.val.reserve((size_t)((e - p) / 10));
    while (p < e) {
        const char* le = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
        if (!le) le = e;
        if (*p != '%') {
            const char* tb[3];
            const char* te[3];
            int nt = 0;
            const char* q = p;
            while (q < le && nt < 3) {
                while (q < le && is_ws(*q)) ++q;
                if (q >= le) break;
                tb[nt] = q;
                while (q < le && !is_ws(*q)) ++q;
                te[nt++] = q;
            }
            if (nt == 3) {
                const int64_t r = parse_int(tb[0], te[0]) - 1, c = parse_int(tb[1], te[1]) - 1;
                if (r < 0 || r >= D || c < 0 || c >= N) {
                    if (ch.err.empty())
                        ch.err = "entry (" + std::to_string(r + 1) + ", " + std::to_string(c + 1) +
                                 ") outside the " + std::to_string(D) + " x " + std::to_string(N) + " header";
                } else {
                    ch.gene.push_back((int32_t)r);
                    ch.cell.push_back((int32_t)c);
                    ch.val.push_back(parse_float(tb[2], te[2]));
                    ch.cmin = std::min(ch.cmin, c);
                    ch.cmax = std::max(ch.cmax, c);
                }
            }
        }
        p = le + 1;
    }
}

// header: skip '%' lines; first other line = rows cols nnz (peek_bgzf_header)
static bool parse_header(const std::vector<char>& t, size_t& pos, int64_t& rows, int64_t& cols, int64_t& nnz) {
    pos = 0;
    while (pos < t.size()) {
        const char* p = t.data() + pos;
        const char* e = t.data() + t.size();
        const char* le = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
        if (!le) le = e;
        const size_t next = (size_t)(le - t.data()) + 1;
        if (*p != '%' && le > p) {
            int64_t v[3];
            int nt = 0;
            const char* q = p;
            while (q < le && nt < 3) {
                while (q < le && is_ws(*q)) ++q;
                if (q >= le) break;
                const char* a = q;
                while (q < le && !is_ws(*q)) ++q;
                v[nt++] = parse_int(a, q);
            }
            pos = next;
            if (nt < 2) return false;
            rows = v[0];
            cols = v[1];
            nnz = nt > 2 ? v[2] : 0;
            return rows > 0 && cols > 0;
        }
        pos = next;
    }
    return false;
}

int read_triplets(const char* path, int threads, int64_t& D, int64_t& N, std::vector<Chunk>& chunks) {
    threads = default_threads(threads);
    std::vector<char> text;
    std::string err;
    if (!load_text(path, threads, text, err)) return fail(MMVAE_E_ARG, err);
    size_t pos;
    int64_t nnz_hdr;
    if (!parse_header(text, pos, D, N, nnz_hdr))
        return fail(MMVAE_E_ARG, std::string("no MatrixMarket size line in ") + path);
    if (N >= INT32_MAX || D >= INT32_MAX) return fail(MMVAE_E_ARG, "matrix dimensions exceed int32");
    // split the body at line boundaries
    const size_t body = text.size() - pos;
    const int nch = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads * 4, body / (1 << 16) + 1));
    std::vector<size_t> cut(nch + 1);
    cut[0] = pos;
    cut[nch] = text.size();
    for (int k = 1; k < nch; ++k) {
        size_t c = pos + body * k / nch;
        c = std::max(c, cut[k - 1]);
        while (c < text.size() && text[c - 1] != '\n') ++c;
        cut[k] = c;
    }
    chunks.assign(nch, Chunk());
    std::atomic<int> next{0};
    parallel_for(threads, threads, [&](int, int64_t, int64_t) {
        for (int k = next++; k < nch; k = next++) parse_chunk(text.data() + cut[k], text.data() + cut[k + 1], D, N, chunks[k]);
    });
    for (auto& c : chunks)
        if (!c.err.empty()) return fail(MMVAE_E_ARG, std::string(path) + ": " + c.err);
    return MMVAE_OK;
}

static int finish_csr(int threads, int64_t N, int64_t D, std::vector<int64_t>& rp, std::vector<int32_t>& col,
                      std::vector<float>& val, mmvae_csr* out);
template <class T> struct RawBuf;
static int finish_rows(int threads, int64_t N, std::vector<int64_t>& rp, int32_t* col, float* val, int64_t& nnz);
static int stream_sorted_csr(const char* path, int threads, mmvae_csr* out);

}  // namespace mmvae_host

using namespace mmvae_host;

extern "C" {

const char* mmvae_host_last_error(void) { return g_err.c_str(); }

void mmvae_free(void* p) { std::free(p); }

void mmvae_csr_free(mmvae_csr* c) {
    if (!c) return;
    std::free(c->rowptr);
    std::free(c->col);
    std::free(c->val);
    c->rowptr = nullptr;
    c->col = nullptr;
    c->val = nullptr;
    c->N = c->D = c->nnz = 0;
}

int mmvae_mtx_read(const char* path, int threads, mmvae_csr* out) {
    if (!path || !out) return fail(MMVAE_E_ARG, "mtx_read: null argument");
    std::memset(out, 0, sizeof(*out));
    threads = default_threads(threads);
    {
        const int src = stream_sorted_csr(path, threads, out);  // column-sorted BGZF: streamed
        if (src != 1) return src;
    }
    int64_t D, N;
    std::vector<Chunk> chunks;
    int rc = read_triplets(path, threads, D, N, chunks);
    if (rc) return rc;
    const int nch = (int)chunks.size();
    // per-chunk column histograms over each chunk's column range
    std::vector<std::vector<int64_t>> cnt(nch);
    parallel_for(threads, nch, [&](int, int64_t a, int64_t b) {
        for (int64_t k = a; k < b; ++k) {
            Chunk& ch = chunks[(size_t)k];
            if (ch.cmax < 0) continue;
            cnt[k].assign((size_t)(ch.cmax - ch.cmin + 1), 0);
            for (int32_t c : ch.cell) cnt[k][(size_t)(c - ch.cmin)]++;
        }
    });
    std::vector<int64_t> rp((size_t)N + 1, 0);
    for (int k = 0; k < nch; ++k)
        for (size_t i = 0; i < cnt[k].size(); ++i) rp[(size_t)chunks[k].cmin + i + 1] += cnt[k][i];
    for (int64_t i = 0; i < N; ++i) rp[(size_t)i + 1] += rp[(size_t)i];
    const int64_t nnz_all = rp[(size_t)N];
    // each chunk's start offset per column = rowptr + entries of earlier chunks (file order)
    {
        std::vector<int64_t> run(rp.begin(), rp.end() - 1);
        for (int k = 0; k < nch; ++k)
            for (size_t i = 0; i < cnt[k].size(); ++i) {
                const size_t c = (size_t)chunks[k].cmin + i;
                const int64_t n = cnt[k][i];
                cnt[k][i] = run[c];
                run[c] += n;
            }
    }
    std::vector<int32_t> col((size_t)nnz_all);
    std::vector<float> val((size_t)nnz_all);
    parallel_for(threads, nch, [&](int, int64_t a, int64_t b) {
        for (int64_t k = a; k < b; ++k) {
            Chunk& ch = chunks[(size_t)k];
            for (size_t e = 0; e < ch.cell.size(); ++e) {
                const int64_t o = cnt[k][(size_t)(ch.cell[e] - ch.cmin)]++;
                col[(size_t)o] = ch.gene[e];
                val[(size_t)o] = ch.val[e];
            }
            std::vector<int32_t>().swap(ch.cell);
            std::vector<int32_t>().swap(ch.gene);
            std::vector<float>().swap(ch.val);
        }
    });
    return finish_csr(threads, N, D, rp, col, val, out);
}

}  // extern "C"

namespace mmvae_host {
// rows strictly increasing in gene: a stable sort + keep-last dedupe of the rows that need it
// (the reference's dense scatter overwrites, mmvae_io.hh:115-123), in place; rp / nnz updated
static int finish_rows(int threads, int64_t N, std::vector<int64_t>& rp, int32_t* col, float* val, int64_t& nnz) {
    std::vector<int64_t> newlen((size_t)N);
    std::atomic<bool> compact{false};
    parallel_for(threads, N, [&](int, int64_t a, int64_t b) {
        std::vector<std::pair<int32_t, int64_t>> tmp;
        std::vector<int32_t> cg;
        std::vector<float> cv;
        for (int64_t r = a; r < b; ++r) {
            const int64_t s = rp[(size_t)r], e = rp[(size_t)r + 1];
            bool ok = true;
            for (int64_t j = s + 1; j < e && ok; ++j) ok = col[(size_t)j] > col[(size_t)j - 1];
            newlen[(size_t)r] = e - s;
            if (ok) continue;
            tmp.clear();
            for (int64_t j = s; j < e; ++j) tmp.emplace_back(col[(size_t)j], j);
            std::stable_sort(tmp.begin(), tmp.end(),
                             [](const std::pair<int32_t, int64_t>& x, const std::pair<int32_t, int64_t>& y) {
                                 return x.first < y.first;
                             });
            cg.clear();
            cv.clear();
            for (size_t i = 0; i < tmp.size(); ++i) {
                if (i + 1 < tmp.size() && tmp[i + 1].first == tmp[i].first) continue;  // keep the last
                cg.push_back(tmp[i].first);
                cv.push_back(val[(size_t)tmp[i].second]);
            }
            for (size_t i = 0; i < cg.size(); ++i) {
                col[(size_t)s + i] = cg[i];
                val[(size_t)s + i] = cv[i];
            }
            if ((int64_t)cg.size() != e - s) compact = true;
            newlen[(size_t)r] = (int64_t)cg.size();
        }
    });
    nnz = rp[(size_t)N];
    if (compact) {
        std::vector<int64_t> np((size_t)N + 1, 0);
        for (int64_t r = 0; r < N; ++r) np[(size_t)r + 1] = np[(size_t)r] + newlen[(size_t)r];
        nnz = np[(size_t)N];
        for (int64_t r = 0; r < N; ++r) {
            std::memmove(col + np[(size_t)r], col + rp[(size_t)r], sizeof(int32_t) * (size_t)newlen[(size_t)r]);
            std::memmove(val + np[(size_t)r], val + rp[(size_t)r], sizeof(float) * (size_t)newlen[(size_t)r]);
        }
        rp.swap(np);
    }
    return MMVAE_OK;
}

static int finish_csr(int threads, int64_t N, int64_t D, std::vector<int64_t>& rp, std::vector<int32_t>& col,
                      std::vector<float>& val, mmvae_csr* out) {
    int64_t nnz = 0;
    finish_rows(threads, N, rp, col.data(), val.data(), nnz);
    out->N = N;
    out->D = D;
    out->nnz = nnz;
    out->rowptr = static_cast<int64_t*>(std::malloc(sizeof(int64_t) * ((size_t)N + 1)));
    out->col = static_cast<int32_t*>(std::malloc(sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1)));
    out->val = static_cast<float*>(std::malloc(sizeof(float) * (size_t)std::max<int64_t>(nnz, 1)));
    if (!out->rowptr || !out->col || !out->val) {
        mmvae_csr_free(out);
        return fail(MMVAE_E_ARG, "out of host memory");
    }
    std::memcpy(out->rowptr, rp.data(), sizeof(int64_t) * ((size_t)N + 1));
    std::memcpy(out->col, col.data(), sizeof(int32_t) * (size_t)nnz);
    std::memcpy(out->val, val.data(), sizeof(float) * (size_t)nnz);
    return MMVAE_OK;
}

// ---- streaming load of a column-sorted BGZF MatrixMarket file ------------------------------
// (the mmutil convention: entries grouped by column = cell, as write_matrix_market_stream and
// 10x-style matrix.mtx.gz files are).  File order is then CSR order, so the file streams straight
// into the cell-major CSR: windows of whole BGZF blocks (64 MB compressed, MMVAE_MTX_WINDOW bytes
// to override) are split into one contiguous block range per worker, and each worker inflates its
// blocks one at a time into a block-sized buffer and parses the complete lines at once, while the
// block is in cache (replaces visit_bgzf_block's inflate-then-scan, mmutil_bgzf_util.hh:53-151).
// A worker's output is its genes and values in file order plus (cell, count) runs; the line cut
// by each range boundary is stitched and parsed serially.  Neither the text (~12 B per entry) nor
// a per-entry cell id is ever stored: peak memory ~ the CSR plus one compressed window.  Returns 1
// (the caller takes the whole-file path) for input that is not BGZF or whose columns are not
// sorted.

// malloc-backed array with uninitialised growth (no zero fill of bytes about to be overwritten)
template <class T>
struct RawBuf {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    RawBuf() = default;
    RawBuf(const RawBuf&) = delete;
    RawBuf& operator=(const RawBuf&) = delete;
    ~RawBuf() { std::free(p); }
    bool reserve(size_t c) {
        if (c <= cap) return true;
        const size_t nc = std::max(c, cap + cap / 2 + 1024);
        T* q = static_cast<T*>(std::realloc(p, nc * sizeof(T)));
        if (!q) return false;
        p = q;
        cap = nc;
        return true;
    }
    T* release() {
        T* q = p;
        p = nullptr;
        n = cap = 0;
        return q;
    }
};

struct Run {
    int32_t cell;
    int64_t count;
};

struct StreamPart {
    RawBuf<int32_t> gene;
    RawBuf<float> val;
    std::vector<Run> runs;
    std::string head, tail;  // text before the range's first newline / after its last
    bool any_nl = false;
    bool ok = true;
    std::string err;
};

// the complete lines of [p, e) into o (file order): '%' lines and lines with < 3 fields skipped,
// as mmutil_bgzf_util.hh:102-127 does
static bool stream_lines(const char* p, const char* e, int64_t D, int64_t N, StreamPart& o) {
    // every entry line takes >= 6 bytes ("1 1 1\n")
    if (!o.gene.reserve(o.gene.n + (size_t)(e - p) / 6 + 1) || !o.val.reserve(o.val.n + (size_t)(e - p) / 6 + 1)) {
        o.err = "out of host memory";
        return false;
    }
    int32_t* gp = o.gene.p;
    float* vp = o.val.p;
    size_t n = o.gene.n;
    int32_t run_cell = o.runs.empty() ? -1 : o.runs.back().cell;
    int64_t run_n = 0;  // entries of run_cell not yet added to its run
    auto flush = [&] {
        if (run_n) o.runs.back().count += run_n;
        run_n = 0;
    };
    while (p < e) {
        // fast path, the common line "gene cell count\n" (unsigned decimal integers, single
        // blanks or tabs): anything else falls through to the general tokenizer below
        {
            const char* q = p;
            uint64_t r = 0, c = 0, x = 0;
            const char* d = q;
            while ((unsigned)(*q - '0') < 10u) r = r * 10 + (uint64_t)(*q++ - '0');
            if (q > d && q - d < 10 && (*q == ' ' || *q == '\t')) {
                ++q;
                d = q;
                while ((unsigned)(*q - '0') < 10u) c = c * 10 + (uint64_t)(*q++ - '0');
                if (q > d && q - d < 10 && (*q == ' ' || *q == '\t')) {
                    ++q;
                    d = q;
                    while ((unsigned)(*q - '0') < 10u) x = x * 10 + (uint64_t)(*q++ - '0');
                    if (q > d && q - d < 16 && *q == '\n' && r >= 1 && (int64_t)r <= D && c >= 1 && (int64_t)c <= N) {
                        gp[n] = (int32_t)(r - 1);
                        vp[n] = (float)x;
                        ++n;
                        if ((int32_t)(c - 1) == run_cell) {
                            ++run_n;
                        } else {
                            flush();
                            o.runs.push_back(Run{(int32_t)(c - 1), 1});
                            run_cell = (int32_t)(c - 1);
                        }
                        p = q + 1;
                        continue;
                    }
                }
            }
        }
        flush();
        const char* le = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
        if (!le) le = e;
        if (*p != '%') {
            const char* tb[3];
            const char* te[3];
            int nt = 0;
            const char* q = p;
            while (q < le && nt < 3) {
                while (q < le && is_ws(*q)) ++q;
                if (q >= le) break;
                tb[nt] = q;
                while (q < le && !is_ws(*q)) ++q;
                te[nt++] = q;
            }
            if (nt == 3) {
                const int64_t r = parse_int(tb[0], te[0]) - 1, c = parse_int(tb[1], te[1]) - 1;
                if (r < 0 || r >= D || c < 0 || c >= N) {
                    o.err = "entry (" + std::to_string(r + 1) + ", " + std::to_string(c + 1) + ") outside the " +
                            std::to_string(D) + " x " + std::to_string(N) + " header";
                    o.gene.n = n;
                    o.val.n = n;
                    return false;
                }
                gp[n] = (int32_t)r;
                vp[n] = parse_float(tb[2], te[2]);
                ++n;
                if (!o.runs.empty() && o.runs.back().cell == (int32_t)c) ++o.runs.back().count;
                else o.runs.push_back(Run{(int32_t)c, 1});
                run_cell = (int32_t)c;
            }
        }
        p = le + 1;
    }
    flush();
    o.gene.n = n;
    o.val.n = n;
    return true;
}

// the streamed buffers handed to `out` as they are (no copy)
static int finish_csr_raw(int threads, int64_t N, int64_t D, std::vector<int64_t>& rp, RawBuf<int32_t>& col,
                          RawBuf<float>& val, mmvae_csr* out) {
    if (!col.reserve(1) || !val.reserve(1)) return fail(MMVAE_E_ARG, "out of host memory");
    int64_t nnz = 0;
    finish_rows(threads, N, rp, col.p, val.p, nnz);
    out->N = N;
    out->D = D;
    out->nnz = nnz;
    out->rowptr = static_cast<int64_t*>(std::malloc(sizeof(int64_t) * ((size_t)N + 1)));
    if (!out->rowptr) return fail(MMVAE_E_ARG, "out of host memory");
    std::memcpy(out->rowptr, rp.data(), sizeof(int64_t) * ((size_t)N + 1));
    out->col = col.release();
    out->val = val.release();
    return MMVAE_OK;
}

static int stream_sorted_csr(const char* path, int threads, mmvae_csr* out) {
    // MMVAE_MTX_PROFILE=1: phase times (read, parallel inflate + parse, stitch + append, rows)
    const bool prof = std::getenv("MMVAE_MTX_PROFILE") != nullptr;
    double tp[4] = {0, 0, 0, 0};
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto since = [](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    };
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return fail(MMVAE_E_ARG, std::string("cannot open ") + path + ": " + std::strerror(errno));
    size_t WIN = (size_t)64 << 20;
    if (const char* ev = std::getenv("MMVAE_MTX_WINDOW")) WIN = std::max<size_t>((size_t)std::atoll(ev), 4096);
    // two window buffers: the next window is read by a helper thread while this one is processed;
    // the partial BGZF block left at a window's end (< 64 KB) moves to just before the next one's
    // bytes (PAD of room), so a window is always one contiguous range
    constexpr size_t PAD = (size_t)128 << 10;
    RawBuf<unsigned char> wbuf[2];
    if (!wbuf[0].reserve(PAD + WIN) || !wbuf[1].reserve(PAD + WIN)) {
        std::fclose(fp);
        return fail(MMVAE_E_ARG, "out of host memory");
    }
    int cb = 0;
    size_t lead = 0;                                       // leftover bytes before wbuf[cb] + PAD
    size_t got = std::fread(wbuf[0].p + PAD, 1, WIN, fp);  // this window's new bytes
    bool header = false, first = true;
    int64_t D = 0, N = 0, nnz_hdr = 0, last_cell = -1;
    std::vector<int64_t> rp;
    RawBuf<int32_t> col;
    RawBuf<float> val;
    std::vector<BgzfBlock> blocks;
    std::string carry;  // the partial line at the end of the previous window
    int rc = MMVAE_OK;
    // one line of text outside every worker's range (a stitched boundary line or the file's last)
    auto single = [&](const std::string& line, StreamPart& sp) -> bool {
        if (line.empty()) return true;
        std::string l = line;
        l.push_back('\n');
        return stream_lines(l.data(), l.data() + l.size(), D, N, sp);
    };
    // entries of the parts, in order, appended to the CSR; false: columns not sorted
    auto append = [&](std::vector<StreamPart*>& parts) -> int {
        size_t tot = col.n;
        std::vector<size_t> off(parts.size() + 1, col.n);
        for (size_t k = 0; k < parts.size(); ++k) {
            if (!parts[k]->err.empty()) return fail(MMVAE_E_ARG, std::string(path) + ": " + parts[k]->err);
            for (const Run& r : parts[k]->runs) {
                if (r.cell < last_cell) return 1;  // not column-sorted: the whole-file path
                last_cell = r.cell;
                rp[(size_t)r.cell + 1] += r.count;
            }
            tot += parts[k]->gene.n;
            off[k + 1] = tot;
        }
        if (!col.reserve(tot) || !val.reserve(tot)) return fail(MMVAE_E_ARG, "out of host memory");
        parallel_for(threads, (int64_t)parts.size(), [&](int, int64_t a, int64_t b) {
            for (int64_t k = a; k < b; ++k) {
                const StreamPart& sp = *parts[(size_t)k];
                if (!sp.gene.n) continue;
                std::memcpy(col.p + off[(size_t)k], sp.gene.p, sp.gene.n * sizeof(int32_t));
                std::memcpy(val.p + off[(size_t)k], sp.val.p, sp.val.n * sizeof(float));
            }
        });
        col.n = val.n = tot;
        return MMVAE_OK;
    };
    for (bool eof = false; !eof && rc == MMVAE_OK;) {
        auto t0 = now();
        unsigned char* const cbuf = wbuf[cb].p + PAD - lead;
        const size_t have = lead + got;
        eof = got == 0;
        size_t got_next = 0;
        std::thread reader;
        if (!eof) reader = std::thread([&] { got_next = std::fread(wbuf[cb ^ 1].p + PAD, 1, WIN, fp); });
        struct Join {
            std::thread& t;
            ~Join() {
                if (t.joinable()) t.join();
            }
        } join_reader{reader};
        size_t used = 0;
        if (!scan_bgzf_window(cbuf, have, blocks, used)) {
            rc = first ? 1 : fail(MMVAE_E_ARG, std::string("corrupt BGZF block in ") + path);
            break;
        }
        if (eof && used != have) {
            rc = fail(MMVAE_E_ARG, std::string("truncated BGZF block at the end of ") + path);
            break;
        }
        auto next_window = [&] {
            if (reader.joinable()) reader.join();
            const size_t left = have - used;
            std::memcpy(wbuf[cb ^ 1].p + PAD - left, cbuf + used, left);
            lead = left;
            got = got_next;
            cb ^= 1;
        };
        if (blocks.empty()) {
            next_window();
            continue;
        }
        size_t skip = 0;  // bytes of the first block taken by the header lines
        if (first) {
            first = false;
            std::vector<char> b0(blocks[0].out_len);
            if (!inflate_raw(cbuf + blocks[0].in_off, blocks[0].in_len, b0.data(), b0.size())) {
                rc = fail(MMVAE_E_ARG, std::string("corrupt BGZF block in ") + path);
                break;
            }
            size_t pos = 0;
            if (!parse_header(b0, pos, D, N, nnz_hdr) || pos > b0.size()) {
                rc = 1;  // no size line in the first block: the whole-file path reports it
                break;
            }
            if (N >= INT32_MAX || D >= INT32_MAX) {
                rc = fail(MMVAE_E_ARG, "matrix dimensions exceed int32");
                break;
            }
            header = true;
            skip = pos;
            rp.assign((size_t)N + 1, 0);
            if (!col.reserve((size_t)std::max<int64_t>(nnz_hdr, 0)) || !val.reserve((size_t)std::max<int64_t>(nnz_hdr, 0))) {
                rc = fail(MMVAE_E_ARG, "out of host memory");
                break;
            }
        }
        tp[0] += since(t0);
        t0 = now();
        const int nw = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, blocks.size()));
        std::vector<StreamPart> part((size_t)nw);
        parallel_for(nw, nw, [&](int, int64_t w0, int64_t w1) {
            std::vector<char> buf;
            for (int64_t w = w0; w < w1; ++w) {
                StreamPart& sp = part[(size_t)w];
                const size_t b0 = blocks.size() * (size_t)w / (size_t)nw, b1 = blocks.size() * (size_t)(w + 1) / (size_t)nw;
                std::string pend;  // a line continued from the previous block of this range
                for (size_t i = b0; i < b1 && sp.ok; ++i) {
                    const BgzfBlock& k = blocks[i];
                    buf.resize(k.out_len);
                    if (!inflate_raw(cbuf + k.in_off, k.in_len, buf.data(), k.out_len)) {
                        sp.ok = false;
                        sp.err = std::string("corrupt BGZF block");
                        break;
                    }
                    const char* t = buf.data();
                    const char* te = t + k.out_len;
                    if (i == 0 && skip) {  // the header (whole lines) is consumed
                        t += skip;
                        sp.any_nl = true;
                    }
                    if (!sp.any_nl) {
                        const char* nl = static_cast<const char*>(std::memchr(t, '\n', (size_t)(te - t)));
                        if (!nl) {
                            sp.head.append(t, (size_t)(te - t));
                            continue;
                        }
                        sp.head.append(t, (size_t)(nl - t));
                        sp.any_nl = true;
                        t = nl + 1;
                    }
                    const char* last = te;
                    while (last > t && last[-1] != '\n') --last;  // complete lines end at last
                    if (last == t) {
                        pend.append(t, (size_t)(te - t));
                        continue;
                    }
                    if (!pend.empty()) {
                        const char* nl = static_cast<const char*>(std::memchr(t, '\n', (size_t)(te - t)));
                        pend.append(t, (size_t)(nl - t + 1));
                        if (!stream_lines(pend.data(), pend.data() + pend.size(), D, N, sp)) sp.ok = false;
                        pend.clear();
                        t = nl + 1;
                    }
                    if (t < last && !stream_lines(t, last, D, N, sp)) sp.ok = false;
                    pend.assign(last, (size_t)(te - last));
                }
                sp.tail = pend;
            }
        });
        tp[1] += since(t0);
        t0 = now();
        // stitch: carry + the first range's head, each range's tail + the next range's head
        std::vector<StreamPart> glue((size_t)nw);
        std::vector<StreamPart*> order;
        for (int w = 0; w < nw; ++w) {
            StreamPart& sp = part[(size_t)w];
            if (!sp.ok && sp.err.empty()) sp.err = "parse error";
            if (!sp.any_nl) {  // the range holds no line end: all of it continues the carry
                carry += sp.head;
                continue;
            }
            carry += sp.head;
            if (!single(carry, glue[(size_t)w])) glue[(size_t)w].ok = false;
            carry = sp.tail;
            order.push_back(&glue[(size_t)w]);
            order.push_back(&sp);
        }
        rc = append(order);
        next_window();
        tp[2] += since(t0);
    }
    std::fclose(fp);
    if (rc == MMVAE_OK && !carry.empty()) {
        StreamPart last;
        if (!single(carry, last)) rc = fail(MMVAE_E_ARG, std::string(path) + ": " + last.err);
        std::vector<StreamPart*> o{&last};
        if (rc == MMVAE_OK) rc = append(o);
    }
    if (rc != MMVAE_OK) return rc;
    if (!header) return 1;
    for (int64_t i = 0; i < N; ++i) rp[(size_t)i + 1] += rp[(size_t)i];
    const auto t0 = now();
    rc = finish_csr_raw(threads, N, D, rp, col, val, out);
    tp[3] = since(t0);
    if (prof)
        std::fprintf(stderr, "mtx stream: read %.3f  inflate+parse %.3f  stitch+append %.3f  rows %.3f s\n", tp[0], tp[1],
                     tp[2], tp[3]);
    return rc;
}
}  // namespace mmvae_host

extern "C" {

int mmvae_mtx_read_dense_t(const char* path, int threads, int64_t* N_out, int64_t* C_out, float** out) {
    if (!path || !N_out || !C_out || !out) return fail(MMVAE_E_ARG, "mtx_read_dense_t: null argument");
    int64_t D, N;
    std::vector<Chunk> chunks;
    int rc = read_triplets(path, threads, D, N, chunks);
    if (rc) return rc;
    float* m = static_cast<float*>(std::calloc((size_t)(N * D), sizeof(float)));
    if (!m) return fail(MMVAE_E_ARG, "out of host memory");
    for (auto& ch : chunks)  // file order: later entries overwrite (mmvae_io.hh:120-121)
        for (size_t e = 0; e < ch.cell.size(); ++e) m[(size_t)ch.cell[e] * (size_t)D + (size_t)ch.gene[e]] = ch.val[e];
    *N_out = N;
    *C_out = D;
    *out = m;
    return MMVAE_OK;
}

int mmvae_csr_save(const char* path, const mmvae_csr* c) {
    if (!path || !c) return fail(MMVAE_E_ARG, "csr_save: null argument");
    // written under a process-unique temporary name and renamed into place: a reader never sees
    // a torn file, and concurrent writers (one per rank) each publish a complete copy
    const std::string tmp = std::string(path) + ".tmp." + std::to_string((long long)getpid());
    FILE* fp = std::fopen(tmp.c_str(), "wb");
    if (!fp) return fail(MMVAE_E_ARG, std::string("cannot write ") + tmp);
    const char magic[8] = {'M', 'M', 'V', 'A', 'E', 'C', 'S', 'R'};
    bool ok = std::fwrite(magic, 1, 8, fp) == 8 && std::fwrite(&c->N, 8, 1, fp) == 1 &&
              std::fwrite(&c->D, 8, 1, fp) == 1 && std::fwrite(&c->nnz, 8, 1, fp) == 1 &&
              std::fwrite(c->rowptr, 8, (size_t)c->N + 1, fp) == (size_t)c->N + 1 &&
              std::fwrite(c->col, 4, (size_t)c->nnz, fp) == (size_t)c->nnz &&
              std::fwrite(c->val, 4, (size_t)c->nnz, fp) == (size_t)c->nnz;
    ok = (std::fclose(fp) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path) != 0) {
        std::remove(tmp.c_str());
        return fail(MMVAE_E_ARG, std::string("short write on ") + path);
    }
    return MMVAE_OK;
}

int mmvae_csr_load(const char* path, mmvae_csr* c) {
    if (!path || !c) return fail(MMVAE_E_ARG, "csr_load: null argument");
    std::memset(c, 0, sizeof(*c));
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return fail(MMVAE_E_ARG, std::string("cannot open ") + path);
    char magic[8];
    bool ok = std::fread(magic, 1, 8, fp) == 8 && std::memcmp(magic, "MMVAECSR", 8) == 0 &&
              std::fread(&c->N, 8, 1, fp) == 1 && std::fread(&c->D, 8, 1, fp) == 1 && std::fread(&c->nnz, 8, 1, fp) == 1 &&
              c->N > 0 && c->nnz >= 0;
    if (ok) {
        c->rowptr = static_cast<int64_t*>(std::malloc(8 * ((size_t)c->N + 1)));
        c->col = static_cast<int32_t*>(std::malloc(4 * (size_t)std::max<int64_t>(c->nnz, 1)));
        c->val = static_cast<float*>(std::malloc(4 * (size_t)std::max<int64_t>(c->nnz, 1)));
        ok = c->rowptr && c->col && c->val &&
             std::fread(c->rowptr, 8, (size_t)c->N + 1, fp) == (size_t)c->N + 1 &&
             std::fread(c->col, 4, (size_t)c->nnz, fp) == (size_t)c->nnz &&
             std::fread(c->val, 4, (size_t)c->nnz, fp) == (size_t)c->nnz;
    }
    // the trailing byte must be the end of the file, and the row pointers a valid CSR of nnz
    // entries with gene ids inside [0, D): a stale or foreign file is rejected, never walked
    ok = ok && std::fgetc(fp) == EOF;
    std::fclose(fp);
    if (ok) ok = c->D > 0 && c->rowptr[0] == 0 && c->rowptr[c->N] == c->nnz;
    for (int64_t i = 0; ok && i < c->N; ++i) ok = c->rowptr[i + 1] >= c->rowptr[i];
    for (int64_t j = 0; ok && j < c->nnz; ++j) ok = c->col[j] >= 0 && c->col[j] < c->D;
    if (!ok) {
        mmvae_csr_free(c);
        return fail(MMVAE_E_ARG, std::string("not a valid CSR cache: ") + path);
    }
    return MMVAE_OK;
}

// ---- ${mtx}.index (mmutil_index.hh:38-190) -------------------------------------------------
// build_mmutil_index: for every column of a column-sorted BGZF MatrixMarket file, the BGZF
// virtual offset (block address << 16 | offset in the block) of its first line, written as gzip
// text "col voff" lines with 0-based columns (write_tuple_stream, io.hh:248-266).  Offsets are
// the reader's bgzf_tell after the previous line (mm_column_indexer_t::eval, :66-86): a line
// that starts at a block boundary is addressed in the next block at offset 0 (bgzf.c:626-665).
int mmvae_mtx_build_index(const char* mtx, const char* index_file) {
    using namespace mmvae_host;
    if (!mtx) return fail(MMVAE_E_ARG, "build_index: null path");
    const std::string idx = (index_file && index_file[0]) ? std::string(index_file) : std::string(mtx) + ".index";
    FILE* fp = std::fopen(mtx, "rb");
    if (!fp) return fail(MMVAE_E_ARG, std::string("cannot open ") + mtx + ": " + std::strerror(errno));
    {
        unsigned char magic[2] = {0, 0};
        const bool gz = std::fread(magic, 1, 2, fp) == 2 && magic[0] == 0x1f && magic[1] == 0x8b;
        std::rewind(fp);
        if (!gz) {
            std::fclose(fp);
            return fail(MMVAE_E_ARG, std::string("This file is not bgzipped: ") + mtx);
        }
    }
    {
        FILE* fe = std::fopen(idx.c_str(), "rb");  // mmutil_index.hh:152-155: an existing index is kept
        if (fe) {
            std::fclose(fe);
            std::fclose(fp);
            return MMVAE_OK;
        }
    }
    // Streamed window by window (64 MB of whole BGZF blocks, MMVAE_MTX_WINDOW to override), like
    // the loader: peak memory is one window and its text, never the whole inflated file.
    size_t WIN = (size_t)64 << 20;
    if (const char* ev = std::getenv("MMVAE_MTX_WINDOW")) WIN = std::max<size_t>((size_t)std::atoll(ev), 4096);
    const int threads = default_threads(0);
    std::vector<unsigned char> cbuf;
    std::vector<BgzfBlock> blocks;
    std::vector<char> text;
    std::string carry;           // the partial last line of the previous window
    size_t have = 0;
    size_t file_base = 0;        // file offset of cbuf[0]
    size_t ubase = 0;            // uncompressed offset of the current window's first block
    int64_t rows = 0, cols = 0, nnz = 0;
    bool have_header = false, first = true;
    int64_t lineno = 0, last_col = 0, last_off = 0, first_off = 0;
    std::vector<std::pair<int64_t, int64_t>> map;
    int rc = MMVAE_OK;
    for (bool eof = false; !eof && rc == MMVAE_OK;) {
        cbuf.resize(have + WIN);
        const size_t r = std::fread(cbuf.data() + have, 1, WIN, fp);
        have += r;
        eof = r == 0;
        size_t used = 0;
        if (!scan_bgzf_window(cbuf.data(), have, blocks, used) || (first && blocks.empty() && have > 0 && eof)) {
            rc = fail(MMVAE_E_ARG, std::string(first ? "This file is not bgzipped: " : "corrupt BGZF block in ") + mtx);
            break;
        }
        first = false;
        if (eof && used != have) {
            rc = fail(MMVAE_E_ARG, std::string("truncated BGZF block at the end of ") + mtx);
            break;
        }
        if (blocks.empty()) continue;
        const size_t total = blocks.back().out_off + blocks.back().out_len;
        text.resize(carry.size() + total);
        std::memcpy(text.data(), carry.data(), carry.size());
        std::atomic<bool> ok{true};
        parallel_for(threads, (int64_t)blocks.size(), [&](int, int64_t a, int64_t bnd) {
            for (int64_t i = a; i < bnd; ++i) {
                const BgzfBlock& k = blocks[(size_t)i];
                if (!inflate_raw(cbuf.data() + k.in_off, k.in_len, text.data() + carry.size() + k.out_off, k.out_len))
                    ok = false;
            }
        });
        if (!ok) {
            rc = fail(MMVAE_E_ARG, std::string("corrupt BGZF block in ") + mtx);
            break;
        }
        // uncompressed offset (absolute) -> virtual offset: the block holding byte u; u at a
        // block's end maps to the next non-empty block at offset 0, past this window to the block
        // that follows it (the EOF marker block at the end of the file)
        std::vector<size_t> starts, addr;
        for (const auto& b : blocks)
            if (b.out_len > 0) {
                starts.push_back(ubase + b.out_off);
                addr.push_back(file_base + b.file_off);
            }
        const size_t wend = ubase + total;
        const bool last_window = eof || (std::feof(fp) && used == have);
        const size_t next_addr = last_window ? file_base + used - 28 : file_base + used;
        size_t bi = 0;
        auto voff = [&](size_t u) -> int64_t {
            if (starts.empty() || u >= wend) return (int64_t)(next_addr << 16);
            while (bi + 1 < starts.size() && starts[bi + 1] <= u) ++bi;
            return (int64_t)((addr[bi] << 16) | (u - starts[bi]));
        };
        // complete lines of carry + this window's text; text index i is uncompressed offset
        // ubase - carry.size() + i
        const size_t tbase = ubase - carry.size();
        size_t nl = text.size();
        while (nl > 0 && text[nl - 1] != '\n') --nl;
        size_t pos = 0;
        while (pos < nl && rc == MMVAE_OK) {
            const char* ls = text.data() + pos;
            const char* le = static_cast<const char*>(std::memchr(ls, '\n', nl - pos));
            const size_t end = (size_t)(le - text.data()) + 1;
            const int64_t line_start_off = last_off;
            last_off = voff(tbase + end);  // bgzf_tell after this line
            pos = end;
            if (le == ls || ls[0] == '%') continue;
            int64_t f[3];
            int nf = 0;
            const char* p = ls;
            while (p < le && nf < 3) {
                while (p < le && is_ws(*p)) ++p;
                const char* q = p;
                while (q < le && !is_ws(*q)) ++q;
                if (q > p) f[nf++] = parse_int(p, q);
                p = q;
            }
            if (!have_header) {
                if (nf < 3) continue;
                rows = f[0];
                cols = f[1];
                nnz = f[2];
                have_header = true;
                first_off = last_off;  // eval_after_header: tell after the size line (:56-64)
                continue;
            }
            if (nf < 3) continue;
            const int64_t col = f[1] - 1;
            if (lineno == 0) {
                last_col = col;
                map.push_back({col, first_off});
            }
            if (col != last_col) {
                if (col < last_col) rc = fail(MMVAE_E_ARG, std::string("MTX must be sorted by columns: ") + mtx);
                map.push_back({col, line_start_off});
                last_col = col;
            }
            ++lineno;
        }
        carry.assign(text.data() + nl, text.size() - nl);
        ubase = wend;
        std::memmove(cbuf.data(), cbuf.data() + used, have - used);
        file_base += used;
        have -= used;
    }
    std::fclose(fp);
    if (rc != MMVAE_OK) return rc;
    if (!carry.empty()) {  // a last line without its newline (not written by bgzip'd mmutil files)
        int64_t f[3];
        int nf = 0;
        const char* p = carry.data();
        const char* le = p + carry.size();
        while (p < le && nf < 3) {
            while (p < le && is_ws(*p)) ++p;
            const char* q = p;
            while (q < le && !is_ws(*q)) ++q;
            if (q > p) f[nf++] = parse_int(p, q);
            p = q;
        }
        if (have_header && nf >= 3 && carry[0] != '%') {
            const int64_t col = f[1] - 1;
            if (lineno == 0) map.push_back({col, first_off});
            else if (col != last_col) {
                if (col < last_col) return fail(MMVAE_E_ARG, std::string("MTX must be sorted by columns: ") + mtx);
                map.push_back({col, last_off});
            }
        }
    }
    (void)rows;
    (void)nnz;
    if (!have_header) return fail(MMVAE_E_ARG, std::string("no MatrixMarket size line in ") + mtx);
    const int64_t lastc = map.empty() ? 0 : map.back().first;
    if (lastc != cols - 1)  // mmutil_index.hh:171-179
        return fail(MMVAE_E_ARG, "Failed to index all the columns: " + std::to_string(lastc) + " < " +
                                     std::to_string(cols - 1) + " (filter out empty columns)");
    const std::string tmp = idx + ".tmp." + std::to_string((long long)getpid());
    gzFile g = gzopen(tmp.c_str(), "wb6");
    if (!g) return fail(MMVAE_E_ARG, "cannot write " + idx);
    std::string line;
    bool wok = true;
    for (const auto& m : map) {
        line = std::to_string((long long)m.first) + " " + std::to_string((long long)m.second) + "\n";
        wok = wok && gzwrite(g, line.data(), (unsigned)line.size()) == (int)line.size();
    }
    wok = (gzclose(g) == Z_OK) && wok;
    if (!wok || std::rename(tmp.c_str(), idx.c_str()) != 0) {
        std::remove(tmp.c_str());
        return fail(MMVAE_E_ARG, "cannot write " + idx);
    }
    return MMVAE_OK;
}

// read_mmutil_index (mmutil_index.hh:192-228): voff per column [0, max col], missing columns
// back-filled with the next column's offset (the reference's loop stops at MaxIdx - 1)
int mmvae_mtx_read_index(const char* index_file, int64_t** voff_out, int64_t* ncol_out) {
    using namespace mmvae_host;
    if (!index_file || !voff_out || !ncol_out) return fail(MMVAE_E_ARG, "read_index: null argument");
    gzFile g = gzopen(index_file, "rb");
    if (!g) return fail(MMVAE_E_ARG, std::string("cannot open ") + index_file);
    std::string buf;
    char chunk[1 << 16];
    int r;
    while ((r = gzread(g, chunk, sizeof(chunk))) > 0) buf.append(chunk, (size_t)r);
    gzclose(g);
    std::vector<std::pair<int64_t, int64_t>> pairs;
    const char* p = buf.data();
    const char* e = p + buf.size();
    while (p < e) {
        char* q;
        const long long c = std::strtoll(p, &q, 10);
        if (q == p) break;
        p = q;
        const long long v = std::strtoll(p, &q, 10);
        if (q == p) break;
        p = q;
        pairs.push_back({c, v});
    }
    if (pairs.empty()) return fail(MMVAE_E_ARG, std::string("empty file ") + index_file);
    int64_t mx = 0;
    for (auto& pr : pairs) mx = std::max<int64_t>(mx, pr.first);
    int64_t* out = static_cast<int64_t*>(std::malloc(sizeof(int64_t) * (size_t)(mx + 1)));
    if (!out) return fail(MMVAE_E_ARG, "out of memory");
    for (int64_t j = 0; j <= mx; ++j) out[j] = 0;  // MISSING_POS = 0 (mmutil_bgzf_util.hh:17)
    for (auto& pr : pairs) out[pr.first] = pr.second;
    for (int64_t j = 0; j < mx - 1; ++j)
        if (out[j] == 0) out[j] = out[j + 1];
    *voff_out = out;
    *ncol_out = mx + 1;
    return MMVAE_OK;
}

// A cell-major CSR as a genes x cells BGZF MatrixMarket file sorted by column (cell), 1-based
// (write_matrix_market_stream, io.hh:189-227): "integer" when every value is integral
int mmvae_mtx_write_csr(const char* path, const mmvae_csr* c) {
    using namespace mmvae_host;
    if (!path || !c || c->N < 1 || c->D < 1) return fail(MMVAE_E_ARG, "mtx_write_csr: bad arguments");
    bool integral = true;
    for (int64_t j = 0; j < c->nnz && integral; ++j) integral = c->val[j] == std::floor(c->val[j]) && std::fabs(c->val[j]) < 1e9f;
    BgzfWriter w;
    if (!w.open(path)) return fail(MMVAE_E_ARG, std::string("cannot write ") + path);
    w.write(std::string("%%MatrixMarket matrix coordinate ") + (integral ? "integer" : "real") + " general\n");
    w.write(std::to_string((long long)c->D) + " " + std::to_string((long long)c->N) + " " +
            std::to_string((long long)c->nnz) + "\n");
    std::string line;
    char num[64];
    for (int64_t i = 0; i < c->N; ++i) {
        const std::string cs = " " + std::to_string((long long)(i + 1)) + " ";
        for (int64_t j = c->rowptr[i]; j < c->rowptr[i + 1]; ++j) {
            line = std::to_string((long long)c->col[j] + 1);
            line += cs;
            if (integral) line += std::to_string((long long)c->val[j]);
            else {
                std::snprintf(num, sizeof(num), "%.9g", (double)c->val[j]);
                line += num;
            }
            line += '\n';
            w.write(line);
        }
    }
    return w.close() ? MMVAE_OK : fail(MMVAE_E_ARG, std::string("write failed: ") + path);
}

int mmvae_mtx_write_ones(const char* path, int64_t N) {
    if (!path || N < 1) return fail(MMVAE_E_ARG, "mtx_write_ones: bad arguments");
    BgzfWriter w;
    if (!w.open(path)) return fail(MMVAE_E_ARG, std::string("cannot write ") + path);
    // write_matrix_market_stream (io.hh:191-227) of a 1 x N all-ones matrix
    w.write("%%MatrixMarket matrix coordinate integer general\n");
    w.write("1 " + std::to_string(N) + " " + std::to_string(N) + "\n");
    std::string line;
    for (int64_t j = 1; j <= N; ++j) {
        line = "1 " + std::to_string(j) + " 1\n";
        w.write(line);
    }
    return w.close() ? MMVAE_OK : fail(MMVAE_E_ARG, std::string("write failed: ") + path);
}

}  // extern "C"
