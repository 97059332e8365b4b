// Shared pieces of the host runtime (libmmvae_host.so): error slot, worker threads, and the
// two compressed writers the reference's outputs use — BGZF for MatrixMarket files
// (obgzf_stream, io.hh:230-242) and plain gzip for the recorder / scores text (ogzstream,
// io.hh:300-331, 545-575).
#pragma once
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace mmvae_host {

extern thread_local std::string g_err;
int fail(int code, const std::string& msg);
int default_threads(int threads);

// BGZF block writer (SAM spec §4.1): <= 64 KiB of input per raw-deflate member with the 'BC'
// extra field, then the 28-byte EOF block.
class BgzfWriter {
   public:
    bool open(const char* path) {
        fp_ = std::fopen(path, "wb");
        buf_.clear();
        return fp_ != nullptr;
    }
    void write(const std::string& s) { write(s.data(), s.size()); }
    void write(const char* p, size_t n) {
        while (n > 0) {
            const size_t take = std::min(n, kBlock - buf_.size());
            buf_.insert(buf_.end(), p, p + take);
            p += take;
            n -= take;
            if (buf_.size() == kBlock) ok_ = flush() && ok_;
        }
    }
    bool close() {
        if (!fp_) return false;
        if (!buf_.empty()) ok_ = flush() && ok_;
        static const unsigned char eof[28] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0, 0, 0xff, 0x06, 0, 0x42, 0x43,
                                              0x02, 0, 0x1b, 0, 0x03, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        ok_ = std::fwrite(eof, 1, 28, fp_) == 28 && ok_;
        ok_ = std::fclose(fp_) == 0 && ok_;
        fp_ = nullptr;
        return ok_;
    }

   private:
    static constexpr size_t kBlock = 65280;
    bool flush() {
        std::vector<unsigned char> out(compressBound((uLong)buf_.size()) + 64);
        z_stream s{};
        if (deflateInit2(&s, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
        s.next_in = reinterpret_cast<unsigned char*>(buf_.data());
        s.avail_in = (uInt)buf_.size();
        s.next_out = out.data() + 18;
        s.avail_out = (uInt)(out.size() - 26);
        const int r = deflate(&s, Z_FINISH);
        const size_t clen = s.total_out;
        deflateEnd(&s);
        if (r != Z_STREAM_END) return false;
        const size_t total = 18 + clen + 8;
        const unsigned char hdr[18] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0, 0, 0xff, 0x06, 0, 'B', 'C', 0x02, 0,
                                       (unsigned char)((total - 1) & 0xff), (unsigned char)((total - 1) >> 8)};
        std::copy(hdr, hdr + 18, out.begin());
        const uLong crc = crc32(crc32(0L, Z_NULL, 0), reinterpret_cast<unsigned char*>(buf_.data()), (uInt)buf_.size());
        unsigned char* t = out.data() + 18 + clen;
        for (int i = 0; i < 4; ++i) t[i] = (unsigned char)((crc >> (8 * i)) & 0xff);
        for (int i = 0; i < 4; ++i) t[4 + i] = (unsigned char)((buf_.size() >> (8 * i)) & 0xff);
        buf_.clear();
        return std::fwrite(out.data(), 1, total, fp_) == total;
    }
    FILE* fp_ = nullptr;
    std::vector<char> buf_;
    bool ok_ = true;
};

// gzip text writer (ogzstream equivalent); path ending in ".gz" is compressed, else plain
class TextWriter {
   public:
    bool open(const std::string& path) {
        gz_ = path.size() > 3 && path.compare(path.size() - 3, 3, ".gz") == 0;
        if (gz_) g_ = gzopen(path.c_str(), "wb6");
        else f_ = std::fopen(path.c_str(), "w");
        return gz_ ? g_ != nullptr : f_ != nullptr;
    }
    void write(const std::string& s) {
        if (gz_) ok_ = gzwrite(g_, s.data(), (unsigned)s.size()) == (int)s.size() && ok_;
        else ok_ = std::fwrite(s.data(), 1, s.size(), f_) == s.size() && ok_;
    }
    bool close() {
        if (gz_ && g_) ok_ = gzclose(g_) == Z_OK && ok_;
        if (!gz_ && f_) ok_ = std::fclose(f_) == 0 && ok_;
        g_ = nullptr;
        f_ = nullptr;
        return ok_;
    }

   private:
    bool gz_ = false, ok_ = true;
    gzFile g_ = nullptr;
    FILE* f_ = nullptr;
};

// std::ostream default float formatting (%g, 6 significant digits), as the reference's
// `ofs << value` writes every recorder / score number (io.hh:310-318, 545-557)
inline std::string fmt_g(float v) {
    char b[32];
    std::snprintf(b, sizeof(b), "%g", (double)v);
    return b;
}

}  // namespace mmvae_host
