// Step-graph cache key (capi.hip mmvae_run) and the rule that makes it rank-invariant.
//
// Plain C++ (no HIP): tests/test_capi_cpu.py compiles it with g++ and checks the derivation
// under differing per-rank batches.
//
// With RCCL calls inside step graphs (MMVAE_COMM_GRAPH=1) every rank must capture — and run
// the capture agreement's all-reduce — at the same steps, so every field of the key must be a
// function of values all ranks share.  The reference's step (mmvae_alg.hh:290-310) has the
// exchange between backward and clip; the global batch n_total, β, update / eval
// and injected noise are the same on every rank by construction of the data-parallel loop.  The
// rank-local inputs were:
//   * the rank's batch size B — required to be n_total / world exactly (checked here, every step:
//     a rank-local error, raised before any collective is issued);
//   * the row-balancing permutation's on/off (perm): a rule over B and the dataset's shape, plus
//     the MMVAE_NO_BALANCE environment — now read once at mmvae_create and max-agreed over the
//     ranks in comm_sync_capacity;
//   * the batch-dependent buffers (ents, gen): sized once for every rank's worst batch
//     (comm_sync_capacity), so they change only at collective calls.
// The cells themselves — which rows, how many nonzeros — never enter the key.
#pragma once
#include <cstdint>
#include <cstring>

namespace mmvae {

struct GraphKey {
    int64_t B = -1, n_total = 0;
    uint32_t beta_bits = 0;
    int update = 0, use_eps = 0, perm = 0;
    const void* ents = nullptr;
    uint64_t gen = 0;
    bool operator==(const GraphKey& o) const {
        return B == o.B && n_total == o.n_total && beta_bits == o.beta_bits && update == o.update &&
               use_eps == o.use_eps && perm == o.perm && ents == o.ents && gen == o.gen;
    }
};

// The row-balancing permutation (balance_rows): fused path, whole 16-row wave blocks, a
// per-cell nonzero table for the dataset, not disabled by MMVAE_NO_BALANCE.
inline bool balance_rule(int64_t B, bool wide, bool nnz_table, bool no_balance) {
    return !wide && B % 16 == 0 && B >= 32 && nnz_table && !no_balance;
}

struct KeyInputs {
    int64_t B = 0, n_total = 0;
    float beta = 0.f;
    bool update = false, use_eps = false;
    bool perm = false;     // balance_rule's outcome for this step
    int world = 1;
    bool comm_graph = false;  // RCCL calls inside the step graphs
    const void* ents = nullptr;
    uint64_t gen = 0;
};

// 0: *k is the step's key.  -1: a step graph with RCCL calls needs B * world == n_total (every
// rank the same slice size, so that B — and with it perm — follows from n_total alone).
inline int derive_graph_key(const KeyInputs& in, GraphKey* k) {
    if (in.comm_graph && in.B * (int64_t)in.world != in.n_total) return -1;
    k->B = in.B;
    k->n_total = in.n_total;
    std::memcpy(&k->beta_bits, &in.beta, 4);
    k->update = in.update;
    k->use_eps = in.use_eps;
    k->perm = in.perm;
    k->ents = in.ents;
    k->gen = in.gen;
    return 0;
}

// The fields every rank must agree on (the capture agreement compares their min and max over the
// ranks: a mismatch makes every rank fall back to eager steps).  ents is rank-local by nature
// (a device pointer) and excluded; it changes only at collective calls.
inline void key_words(const GraphKey& k, int64_t w[6]) {
    w[0] = k.B;
    w[1] = k.n_total;
    w[2] = (int64_t)k.beta_bits;
    w[3] = k.update | (k.use_eps << 1) | (k.perm << 2);
    w[4] = (int64_t)k.gen;
    w[5] = 0;
}

}  // namespace mmvae
