// Shared device helpers for the mmvae HIP engine (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define MMVAE_DEV __device__ __forceinline__

// the per-step batch entry lists as the tile kernels read them (format: tiles.hpp ListEntries)
struct EntList {
    const uint32_t* w;
    int64_t xoff;  // word offset of the float values; 0: counts in the entry word
};
#define MMVAE_HOSTDEV __host__ __device__ __forceinline__

// ---------------------------------------------------------------------------------------
// MFMA policy: both policies produce 16x16 f32 tiles with the same C/D layout
//   col = lane & 15, row = 4 * (lane >> 4) + reg       (cdna_hip_programming.md §3)
// A[row][k] / B[k][col]: lane supplies row/col (lane & 15) and EPL consecutive k starting
// at KSTEP * s + EPL * (lane >> 4).
// ---------------------------------------------------------------------------------------
template <class T> struct MM;

// Split-bf16 operands ("x3", the fp32-accurate mode): every GEMM operand v is held as two bf16
// planes hi = bf16(v), lo = bf16(v - hi) (|v - hi - lo| <= 2^-16 |v|), and a product is
// accumulated in f32 as lo*hi + hi*lo + hi*hi — three bf16 MFMAs (16x16x32: 16 cycles each)
// for the 8 cycles-per-4-k of the exact f32 MFMA (16x16x4: 32 cycles per 4 k).  The lo planes
// sit at a constant element offset `plane` from the hi planes in HBM and LDS.
struct X3 {};
template <class P> struct Elem { typedef P type; };   // storage element of an operand plane
template <> struct Elem<X3> { typedef __bf16 type; };
template <class P> struct IsX3 { static constexpr bool value = false; };
template <> struct IsX3<X3> { static constexpr bool value = true; };

template <> struct MM<float> {
    static constexpr int KSTEP = 4, EPL = 1;
    typedef float frag;
    static MMVAE_DEV frag load(const float* p) { return *p; }
    static MMVAE_DEV frag load(const float* p, int64_t) { return *p; }
    static MMVAE_DEV f32x4 mma(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static MMVAE_DEV frag zero() { return 0.f; }
    static MMVAE_DEV frag load_f32(const float* p) { return *p; }
};

template <> struct MM<__bf16> {
    static constexpr int KSTEP = 32, EPL = 8;
    typedef bf16x8 frag;
    static MMVAE_DEV frag load(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
    static MMVAE_DEV frag load(const __bf16* p, int64_t) { return *reinterpret_cast<const bf16x8*>(p); }
    static MMVAE_DEV f32x4 mma(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
    // 8 consecutive f32 (16-byte aligned) -> one bf16 fragment (v_cvt_pk_bf16_f32)
    static MMVAE_DEV frag load_f32(const float* p) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        frag f;
        f[0] = (__bf16)a.x; f[1] = (__bf16)a.y; f[2] = (__bf16)a.z; f[3] = (__bf16)a.w;
        f[4] = (__bf16)b.x; f[5] = (__bf16)b.y; f[6] = (__bf16)b.z; f[7] = (__bf16)b.w;
        return f;
    }
    static MMVAE_DEV frag zero() {
        frag z;
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] = (__bf16)0.f;
        return z;
    }
};

// hi / lo split of one f32 (round-to-nearest-even bf16, v_cvt_pk_bf16_f32)
MMVAE_DEV __bf16 bf_hi(float v) { return (__bf16)v; }
MMVAE_DEV __bf16 bf_lo(float v, __bf16 hi) { return (__bf16)(v - (float)hi); }

template <> struct MM<X3> {
    static constexpr int KSTEP = 32, EPL = 8;
    struct frag {
        bf16x8 h, l;
    };
    static MMVAE_DEV frag load(const __bf16* p, int64_t plane) {
        return frag{*reinterpret_cast<const bf16x8*>(p), *reinterpret_cast<const bf16x8*>(p + plane)};
    }
    static MMVAE_DEV f32x4 mma(frag a, frag b, f32x4 c) {
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, c, 0, 0, 0);
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, c, 0, 0, 0);
    }
    // 8 consecutive f32 (16-byte aligned) -> split fragment
    static MMVAE_DEV frag load_f32(const float* p) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        frag f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            f.h[i] = bf_hi(v[i]);
            f.l[i] = bf_lo(v[i], f.h[i]);
        }
        return f;
    }
    static MMVAE_DEV frag zero() {
        frag z;
#pragma unroll
        for (int i = 0; i < 8; ++i) z.h[i] = z.l[i] = (__bf16)0.f;
        return z;
    }
};

// fp8 e4m3 operands (BASELINE configs[4]: the decoder logit GEMM z W_dec^T of passes A, B, C):
// v_mfma_f32_16x16x32_fp8_fp8, 8 e4m3 values per lane (one 64-bit register pair), f32
// accumulate.  z is converted from f32 as the fragment is loaded; W_dec is stored pre-scaled by a
// power of two (amax -> the top of the e4m3 range, k_pack_w8) and the accumulator is unscaled.
struct F8 {};
template <> struct Elem<F8> { typedef uint8_t type; };
template <> struct MM<F8> {
    static constexpr int KSTEP = 32, EPL = 8;
    typedef long frag;
    static MMVAE_DEV frag load(const uint8_t* p) { return *reinterpret_cast<const long*>(p); }
    static MMVAE_DEV frag load(const uint8_t* p, int64_t) { return *reinterpret_cast<const long*>(p); }
    static MMVAE_DEV f32x4 mma(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
    }
    // 8 consecutive f32 (16-byte aligned) -> one e4m3 fragment (v_cvt_pk_fp8_f32, RNE)
    static MMVAE_DEV frag load_f32(const float* p) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        int lo = __builtin_amdgcn_cvt_pk_fp8_f32(a.x, a.y, 0, false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(a.z, a.w, lo, true);
        int hi = __builtin_amdgcn_cvt_pk_fp8_f32(b.x, b.y, 0, false);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(b.z, b.w, hi, true);
        return (long)(uint32_t)lo | ((long)(uint32_t)hi << 32);
    }
    static MMVAE_DEV frag zero() { return 0; }
};
template <class P> struct IsF8 { static constexpr bool value = false; };
template <> struct IsF8<F8> { static constexpr bool value = true; };
// policies of the GEMMs that stay bf16 in the fp8 mode (encoder, dz): the mode's own otherwise
template <class P> struct Bf16If8 { typedef P type; };
template <> struct Bf16If8<F8> { typedef __bf16 type; };

// ---------------------------------------------------------------------------------------
// LDS-DMA staging (global_load_lds_dwordx4): the LDS destination is wave-uniform base +
// 16 * lane, so tiles are staged lane-linear and the bank swizzle is applied on the SOURCE
// address.  Image of a [rows][RB-byte] tile: 16-byte chunk c of row r lives at chunk
// c ^ ((r >> 1) & (RB/16 - 1)) — conflict-free for the 16-row MFMA fragment reads
// (ds_read_b128 lane groups, MI355X_MICROARCH.md §LDS).
// ---------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
MMVAE_DEV void glds16(const void* g, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((glb_void_t*)g, (lds_void_t*)lds_wave_base, 16, 0, 0);
}
// diagnostic in-kernel stamp (shader clock); only in MMVAE_DBG-gated diagnostic paths
// constant-rate (100 MHz) clock shared by all CUs, and this wave's placement (diagnostics)
MMVAE_DEV uint64_t realtime_now() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
// xcc << 16 | se << 12 | cu << 4 | simd  (HW_REG_HW_ID = 4, HW_REG_XCC_ID = 20)
MMVAE_DEV uint32_t wave_place() {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xf;
    return (xcc << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 8) & 15) << 4) | ((hw >> 4) & 3);
}
MMVAE_DEV uint64_t stamp_now() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
MMVAE_DEV void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Workgroup barrier that completes this wave's LDS traffic but leaves global loads in flight
// (a __syncthreads() would drain vmcnt(0), exposing the latency of prefetches issued before it).
// Any LDS-DMA that the next phase reads must be retired (vm_wait_all) before calling it.
MMVAE_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <int RB> MMVAE_DEV int swz_off(int row, int byte) {
    constexpr int NCH = RB / 16;
    // 64-byte rows (4 chunks): rows r and r + 8 of a transposed read (tr_frag) share their 256-byte
    // bank window, so bit 3 of the row selects the other chunk pair; the 16-lane ds_read_b128 row
    // reads stay conflict-free with it
    // 128-byte rows (8 chunks): x = row bit 3 -> chunk bit 1, row bit 1 -> chunk bit 2 — found by
    // exhaustive search over linear swizzles: the ds_read_b128 row reads (lane groups of 16) and
    // the transposed 8-byte reads of rows r .. r + 3 and r + 8 .. r + 11 are both conflict-free
    const int x = NCH == 4 ? (((row >> 1) & 1) | ((row >> 2) & 2))
                : NCH == 8 ? ((((row >> 3) & 1) << 1) | (((row >> 1) & 1) << 2))
                           : ((row >> 1) & (NCH - 1));
    return row * RB + (((byte >> 4) ^ x) << 4) + (byte & 15);
}

// MFMA 16x16x32 B fragment of a k-by-column block read TRANSPOSED from a swizzled row-major
// [rows][RB-byte] 16-bit image (the image another GEMM reads row-wise with ds_read_b128):
// k = rows r0 + 8 (lane >> 4) .. + 7, column c0 + (lane & 15).  Two ds_read_b64_tr_b16: per
// 16-lane group, lane 4q + p addresses row q of a 4-row block at columns 4p .. 4p + 3 and lane i
// receives column i of the 4 rows (cdna_hip_programming.md T10).  The 8-byte pieces stay whole
// under swz_off's 16-byte chunk XOR.  EXEC must be all ones.
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
template <int RB> MMVAE_DEV bf16x8 tr_frag(const char* img, int r0, int c0, int lane = (int)threadIdx.x & 63) {
    const int row = r0 + 8 * (lane >> 4) + ((lane >> 2) & 3);
    const int byte = (c0 + 4 * (lane & 3)) * 2;
    typedef __attribute__((address_space(3))) bf16x4 lds_v4;
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(img + swz_off<RB>(row, byte)));
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(img + swz_off<RB>(row + 4, byte)));
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
// 16-bit dz-GEMM A operand of the decoder backward passes (NB pass B pq, vMF pass 1 da), stored
// per 16-gene block as [16 genes][16 rows] bf16 (blocks BS bytes apart; the x3 lo plane at a
// fixed offset after the hi plane): the epilogue writes a lane's row pair of one gene as one
// 32-bit word per plane, and the dz GEMM reads the MFMA A fragment (row lane & 15, genes
// k0 + 8 (lane >> 4) .. + 7) transposed with two ds_read_b64_tr_b16 per plane.  EXEC must be
// all ones.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
MMVAE_DEV uint32_t pk_bf16(float a, float b) { return __builtin_bit_cast(uint32_t, bf16x2{(__bf16)a, (__bf16)b}); }
// (bytes; a gene's 8-byte row quads XOR-swizzled by (g >> 2) & 3: the epilogue's row-pair stores
// go from 4-way to 2-way bank conflicts (free for ds_write_b32) and the transposed reads of genes
// g and g + 8 from 2-way to none — MI355X_MICROARCH.md LDS bank table)
template <int BS = 2048> MMVAE_DEV int pqt_off(int g, int r) {
    return (g >> 4) * BS + (g & 15) * 32 + (((r >> 2) ^ ((g >> 2) & 3)) << 3) + (r & 3) * 2;
}
template <int BS = 2048> MMVAE_DEV bf16x8 pqt_frag(const char* img, int k0, int lane = (int)threadIdx.x & 63) {
    const int k = k0 + 8 * (lane >> 4) + ((lane >> 2) & 3), r = 4 * (lane & 3);
    typedef __attribute__((address_space(3))) bf16x4 lds_v4;
    const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(img + pqt_off<BS>(k, r)));
    const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4*)(img + pqt_off<BS>(k + 4, r)));
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
// a row pair (r, r + 1) of one gene into the transposed image: hi plane word, and for the split
// (x3) operand the lo plane word PO bytes after it
template <int BS, bool SPLIT> MMVAE_DEV void pqt_put(char* img, int PO, int g, int r, float a, float b) {
    char* q = img + pqt_off<BS>(g, r);
    const uint32_t hp = pk_bf16(a, b);
    *reinterpret_cast<uint32_t*>(q) = hp;
    if constexpr (SPLIT) {
        typedef float fp2 __attribute__((ext_vector_type(2)));
        const fp2 lo = fp2{a, b} - fp2{__uint_as_float(hp << 16), __uint_as_float(hp & 0xffff0000u)};
        *reinterpret_cast<uint32_t*>(q + PO) = pk_bf16(lo.x, lo.y);
    }
}

template <class P, int RB> struct TrFrag;
// (lane: threadIdx.x & 63, or a kernel's per-tile opaque copy of it — see k_dec_nb D3)
template <int RB> struct TrFrag<__bf16, RB> {
    static MMVAE_DEV bf16x8 load(const char* img, int r0, int c0, int, int lane = (int)threadIdx.x & 63) {
        return tr_frag<RB>(img, r0, c0, lane);
    }
};
template <int RB> struct TrFrag<X3, RB> {  // hi and lo planes, plane_bytes apart
    static MMVAE_DEV MM<X3>::frag load(const char* img, int r0, int c0, int plane_bytes, int lane = (int)threadIdx.x & 63) {
        return MM<X3>::frag{tr_frag<RB>(img, r0, c0, lane), tr_frag<RB>(img + plane_bytes, r0, c0, lane)};
    }
};

template <class T> MMVAE_DEV T to_t(float v);
template <> MMVAE_DEV float to_t<float>(float v) { return v; }
template <> MMVAE_DEV __bf16 to_t<__bf16>(float v) { return (__bf16)v; }
// one f32 -> e4m3 byte (v_cvt_pk_fp8_f32, round to nearest even)
template <> MMVAE_DEV uint8_t to_t<uint8_t>(float v) {
    return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xff);
}

// ---------------------------------------------------------------------------------------
// Scalar math.  fast exp/log/rcp map to v_exp_f32 / v_log_f32 / v_rcp_f32 (quarter rate).
// ---------------------------------------------------------------------------------------
// Raw v_exp_f32 / v_log_f32 (base 2) — no denormal range fix-ups: every call site feeds
// normal inputs (log args >= 1e-4) or tolerates a flushed tiny exp result.
MMVAE_DEV float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
MMVAE_DEV float flog2(float x) { return __builtin_amdgcn_logf(x); }
MMVAE_DEV float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
MMVAE_DEV float flog(float x) { return __builtin_amdgcn_logf(x) * 0.6931471805599453f; }
MMVAE_DEV float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

// log(1 + r) for r >= 0, accurate for small r (series below 1e-2, else log(1+r): rel err <= 6e-6)
// Both candidates are pinned with an empty asm so the compiler emits v_cndmask instead of
// an exec-masked if/else around the v_log (which costs two divergent paths per element).
MMVAE_DEV float log1p_pos(float r) {
    float series = r * (1.f - r * (0.5f - r * (0.33333334f - r * (0.25f - r * 0.2f))));
    float lg = flog(1.f + r);
    asm volatile("" : "+v"(series), "+v"(lg));
    return (r < 1e-2f) ? series : lg;
}

// torch softplus(beta=1, threshold=20) and its backward factor, branch free:
//   sp = max(u, 0) + log1p(exp(-|u|))    (== u in fp32 for u > 20, the threshold branch)
//   sig = 1 / (1 + exp(-u))             (== 1 in fp32 for u > 20)
MMVAE_DEV float softplus_sig(float u, float& sig) {
    const float e = fexp(-fabsf(u));
    const float r = frcp(1.f + e);
    sig = (u >= 0.f) ? r : e * r;
    return fmaxf(u, 0.f) + log1p_pos(e);
}

// clamp(sp, 1e-4, 1e4) as one v_med3_f32 (nb.hh:459)
MMVAE_DEV float clamp_nu(float sp) { return __builtin_amdgcn_fmed3f(sp, 1e-4f, 1e4f); }

// ---------------------------------------------------------------------------------------
// Packed f32 pairs (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32): one issue covers two
// elements, which halves the issue cost of a VALU-issue-bound loop run by one wave per SIMD.
// ---------------------------------------------------------------------------------------
#ifndef MMVAE_F2_SCALAR
typedef float f2 __attribute__((ext_vector_type(2)));
MMVAE_DEV f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
#else
// the same row-pair code as two scalar f32 streams (v_fma_f32 / v_mul_f32 / v_add_f32)
struct f2 {
    float x, y;
    MMVAE_DEV float& operator[](int i) { return i ? y : x; }
    MMVAE_DEV float operator[](int i) const { return i ? y : x; }
    MMVAE_DEV f2& operator+=(f2 o) { x += o.x; y += o.y; return *this; }
    MMVAE_DEV f2& operator-=(f2 o) { x -= o.x; y -= o.y; return *this; }
    MMVAE_DEV f2& operator*=(f2 o) { x *= o.x; y *= o.y; return *this; }
};
MMVAE_DEV f2 operator+(f2 a, f2 b) { return f2{a.x + b.x, a.y + b.y}; }
MMVAE_DEV f2 operator-(f2 a, f2 b) { return f2{a.x - b.x, a.y - b.y}; }
MMVAE_DEV f2 operator*(f2 a, f2 b) { return f2{a.x * b.x, a.y * b.y}; }
MMVAE_DEV f2 operator+(f2 a, float b) { return f2{a.x + b, a.y + b}; }
MMVAE_DEV f2 operator-(f2 a, float b) { return f2{a.x - b, a.y - b}; }
MMVAE_DEV f2 operator*(f2 a, float b) { return f2{a.x * b, a.y * b}; }
MMVAE_DEV f2 operator+(float a, f2 b) { return f2{a + b.x, a + b.y}; }
MMVAE_DEV f2 operator-(float a, f2 b) { return f2{a - b.x, a - b.y}; }
MMVAE_DEV f2 operator*(float a, f2 b) { return f2{a * b.x, a * b.y}; }
MMVAE_DEV f2 operator-(f2 a) { return f2{-a.x, -a.y}; }
MMVAE_DEV f2 fma2(f2 a, f2 b, f2 c) { return f2{fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)}; }
#endif
MMVAE_DEV f2 splat2(float v) { return f2{v, v}; }

// Dense NB terms of two (cell, gene) elements at x = 0 (nb.hh:456-459, 518-528) — nb_nu2 is its
// overdispersion part, shared with the sparse pass's entry pairs (nb_kernels.hip pass B):
//   nu = clamp(softplus(u)), nup = nu + 1e-4, sgm = d nu / d u (0 where the clamp bites),
//   lg2 = log2((mu + nup) / nup)  (log2 units),  q = -mu / (mu + nup).
// Five transcendentals per element: exp(-|u|), 1/(1+e), log2(1+e), 1/(nup (mu+nup)), log2(s/nup).
// softplus' log1p uses the rounding-corrected form log1p(a) = log(z) - ((z - 1) - a) / z with
// z = fl(1 + a) (exact z - 1): accurate for small a, as torch's log1p.  lg2 is the reference's
// own cancelling difference log(mu + nu) - log(nu) (nb.hh:527), to the same absolute error.
MMVAE_DEV void nb_nu2(f2 u, f2& nup, f2& sgm) {
    constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
    f2 e, r, l;
    e.x = fexp2(-fabsf(u.x) * L2E);
    e.y = fexp2(-fabsf(u.y) * L2E);
    const f2 z = e + 1.f;
    r.x = frcp(z.x);
    r.y = frcp(z.y);
    l.x = flog2(z.x);
    l.y = flog2(z.y);
    const f2 sp = f2{fmaxf(u.x, 0.f), fmaxf(u.y, 0.f)} + fma2(l, splat2(LN2), -(((z - 1.f) - e) * r));
    const f2 nu = f2{clamp_nu(sp.x), clamp_nu(sp.y)};
    const f2 er = e * r;  // sigmoid(u) for u < 0
    sgm.x = (nu.x == sp.x) ? ((u.x >= 0.f) ? r.x : er.x) : 0.f;
    sgm.y = (nu.y == sp.y) ? ((u.y >= 0.f) ? r.y : er.y) : 0.f;
    nup = nu + 1e-4f;
}
MMVAE_DEV void nb_dense2(f2 mu, f2 u, f2& nup, f2& lg2, f2& q, f2& sgm) {
    nb_nu2(u, nup, sgm);
    const f2 sv = mu + nup;
    const f2 ns = nup * sv;
    f2 rr;
    rr.x = frcp(ns.x);
    rr.y = frcp(ns.y);
    const f2 rsv = nup * rr;          // 1 / (mu + nup)
    const f2 zz = sv * (sv * rr);     // (mu + nup) / nup
    lg2.x = flog2(zz.x);
    lg2.y = flog2(zz.y);
    q = -mu * rsv;
}

// accurate torch softplus (libm log1p/exp), for per-row / per-gene scalars
MMVAE_DEV float softplus_acc(float u) { return (u > 20.f) ? u : log1pf(expf(u)); }

MMVAE_DEV float dsoftplus(float u) { return (u > 20.f) ? 1.f : 1.f / (1.f + expf(-u)); }

// ---------------------------------------------------------------------------------------
// Gamma-function terms of the NB likelihood for a count x > 0 and overdispersion nup > 0:
//   lgd = lgamma(nup) + lgamma(x + 1) - lgamma(nup + x)      (nb.hh:522-523)
//   dgd = digamma(nup) - digamma(nup + x)                    (its d/d nup)
// Counts 1..8 (the bulk of single-cell data) use the exact finite product / sum with one log
// and one reciprocal (x! from the caller's LDS table ftab[0..8]).  Everything else shifts each argument below 8 up by 8 (branch free:
// P = v(v+1)..(v+7) and S = P'/P = sum 1/(v+i) by the product rule) and evaluates Stirling's
// series and the digamma asymptotic series at z >= 8 (truncation < 1e-9 relative), sharing
// log z and 1/z between the two.
// ---------------------------------------------------------------------------------------
struct GammaAt {
    float lg, dg;  // lgamma(v), digamma(v)
};
MMVAE_DEV GammaAt gamma_at(float v, bool need_dg) {
    float P = v, Pd = 1.f;
#pragma unroll
    for (int i = 1; i < 8; ++i) {
        const float a = v + (float)i;
        Pd = fmaf(Pd, a, P);
        P *= a;
    }
    const bool sh = v < 8.f;
    const float z = sh ? v + 8.f : v;
    const float lz = flog(z), r = frcp(z), r2 = r * r;
    const float lP = sh ? flog(P) : 0.f;
    GammaAt o;
    o.lg = (z - 0.5f) * lz - z + 0.91893853320467274f +
           r * (0.083333333f - r2 * (0.0027777778f - r2 * 0.00079365079f)) - lP;
    o.dg = 0.f;
    if (need_dg) {
        const float S = sh ? Pd * frcp(P) : 0.f;
        o.dg = lz - 0.5f * r - r2 * (0.083333333f - r2 * (0.0083333333f - r2 * 0.0039682540f)) - S;
    }
    return o;
}

// NF: the largest count on the finite-product path (8; 4 in the f32 mode, whose pass B already
// spills at 256 VGPRs and runs slower with the longer product)
template <int NF = 8>
MMVAE_DEV void nb_gamma_terms(float nup, float x, float& lgd, float& dgd, const float* ftab) {
    // counts up to 8: P <= (nup + 7)^8 <= ~1e32 for the clamped nup <= 1e4 + 1e-4, x! <= 40320 exact
    if (x <= (float)NF && x == floorf(x)) {
        float P = 1.f, Pd = 0.f;
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const bool on = (float)i < x;
            const float a = on ? nup + (float)i : 1.f;
            Pd = on ? fmaf(Pd, a, P) : Pd;
            P *= a;
        }
        const float rP = frcp(P);
        lgd = flog(ftab[(int)x] * rP);  // log(x!) - log(nup (nup+1) .. (nup+x-1))
        dgd = -Pd * rP;         // -sum 1/(nup+i)
    } else {
        const GammaAt a = gamma_at(nup, true), b = gamma_at(nup + x, true), c = gamma_at(x + 1.f, false);
        lgd = a.lg + c.lg - b.lg;
        dgd = a.dg - b.dg;
    }
}

// nb_gamma_terms of two counts that are integers in 0..8 (0: lgd = dgd = 0), as packed pairs.
// Factor i of the finite product is nup + i while i < x, else 1 — on_i = clamp(x - i, 0, 1) is one
// v_pk_add_f32 with the clamp modifier, a_i = on_i (nup + i) + (1 - on_i) — so both counts of a
// pair share every instruction instead of one select chain per count.  x0 / x1: the counts as ints.
#ifndef MMVAE_F2_SCALAR
MMVAE_DEV f2 clamp01_add2(f2 x, float c) {  // min(max(x + c, 0), 1) per half, c wave-uniform
    f2 o;  // (a 64-bit SGPR pair operand whose low word, c, feeds both halves: op_sel_hi)
    const uint64_t cp = (uint64_t)__float_as_uint(c);
    asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] clamp" : "=v"(o) : "v"(x), "s"(cp));
    return o;
}
#else
MMVAE_DEV f2 clamp01_add2(f2 x, float c) {
    return f2{fminf(fmaxf(x.x + c, 0.f), 1.f), fminf(fmaxf(x.y + c, 0.f), 1.f)};
}
#endif
MMVAE_DEV void nb_gamma_terms2(f2 nup, f2 x, int x0, int x1, f2& lgd, f2& dgd, const float* ftab) {
    constexpr float LN2 = 0.6931471805599453f;
    f2 P = splat2(1.f), Pd = splat2(0.f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const f2 on = clamp01_add2(x, -(float)i);
        const f2 a = fma2(on, nup + (float)i, 1.f - on);
        Pd = fma2(Pd, a, on * P);
        P = P * a;
    }
    f2 rP, l;
    rP.x = frcp(P.x);
    rP.y = frcp(P.y);
    const f2 t = f2{ftab[x0], ftab[x1]} * rP;  // x! / (nup (nup+1) .. (nup+x-1))
    l.x = flog2(t.x);
    l.y = flog2(t.y);
    lgd = l * LN2;
    dgd = -Pd * rP;
}

// ---------------------------------------------------------------------------------------
// Wave64 reductions
// ---------------------------------------------------------------------------------------
// sum over the four 16-lane row groups (lanes l, l^16, l^32, l^48), result in every lane
MMVAE_DEV float sum_rowgroups(float v) {
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// four quantities summed over the four row groups at once (transposed butterfly: 3 swaps,
// 3 adds); lane group g = lane >> 4 receives the total of quantity g
MMVAE_DEV float sum_rowgroups4(float a0, float a1, float a2, float a3) {
    const auto s02 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a2), false, false);
    const auto s13 = __builtin_amdgcn_permlane32_swap(__float_as_uint(a1), __float_as_uint(a3), false, false);
    const float b02 = __uint_as_float(s02[0]) + __uint_as_float(s02[1]);  // halves: a0 | a2 over g, g+2
    const float b13 = __uint_as_float(s13[0]) + __uint_as_float(s13[1]);  // halves: a1 | a3
    const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(b02), __float_as_uint(b13), false, false);
    return __uint_as_float(t[0]) + __uint_as_float(t[1]);
}

// two quantities: lanes 0-31 receive the total of a0, lanes 32-63 that of a1
MMVAE_DEV float sum_rowgroups2(float a0, float a1) {
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a1), false, false);
    const float b = __uint_as_float(s[0]) + __uint_as_float(s[1]);
    const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(b), __float_as_uint(b), false, false);
    return __uint_as_float(t[0]) + __uint_as_float(t[1]);
}

MMVAE_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
MMVAE_DEV double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---------------------------------------------------------------------------------------
// Philox4x32-10 counter RNG + Box-Muller: eps(seed, step, row, k) ~ N(0,1).  Keyed by the
// GLOBAL row so data-parallel shards draw the same noise as a single-GPU run.
// ---------------------------------------------------------------------------------------
MMVAE_DEV void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// the overdispersion noise's lanes: NU_LANE + r, disjoint from the latent lanes k < 2^31 at any K
constexpr uint32_t NU_LANE = 0x80000000u;
MMVAE_DEV float philox_normal(uint64_t seed, uint64_t step, uint64_t row, uint32_t k) {
    uint32_t c[4] = {(uint32_t)(k >> 1), (uint32_t)row, (uint32_t)(row >> 32) ^ (uint32_t)step,
                     (uint32_t)(step >> 32)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float u1 = ((c[0] >> 8) + 1) * (1.f / 16777217.f);  // (0,1]
    const float u2 = (c[1] >> 8) * (1.f / 16777216.f);        // [0,1)
    // Box-Muller on the hardware transcendentals: v_sin / v_cos take the angle in revolutions
    // (sin(2 pi u2) with no range reduction), v_log is log2
    const float r = __builtin_amdgcn_sqrtf(-2.f * 0.6931471805599453f * __builtin_amdgcn_logf(u1));
    return r * ((k & 1) ? __builtin_amdgcn_sinf(u2) : __builtin_amdgcn_cosf(u2));
}
