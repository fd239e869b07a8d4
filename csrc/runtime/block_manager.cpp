// block_manager.cpp — paged-KV block allocator with automatic prefix caching (native runtime).
//
// Same semantics as engine/kv_cache.py::PyBlockManager (which remains the CPU-only fallback):
//   * block 0 is reserved (target of padded graph rows), free list of the rest;
//   * refcounted blocks; a FULL block is registered under hash(parent_hash, its tokens);
//   * match_prefix walks a prompt block by block through the hash table (never the whole
//     prompt: one token is left to compute), bumping refcounts;
//   * released cached blocks stay resident, evicted LRU only when the free list is empty.
// Hash: 128-bit FNV-1a variant over (parent hash, token ids) — collisions are astronomically
// unlikely at 2^128 and a match is additionally verified against the stored token ids.
#include "block_manager.h"

using mxrt::BM;
using mxrt::H128;

extern "C" {

void* mxrt_bm_new(int num_blocks, int block_size, int prefix_cache) {
    return new BM(num_blocks, block_size, prefix_cache != 0);
}
void mxrt_bm_free(void* h) { delete (BM*)h; }
void mxrt_bm_set_lifo(void* h, int on) { ((BM*)h)->lifo = on != 0; }
int mxrt_bm_num_free(void* h) { return ((BM*)h)->num_free(); }

// allocate n blocks into out; returns 0 on success, -1 if not enough (nothing allocated)
int mxrt_bm_allocate(void* h, int n, int32_t* out) { return ((BM*)h)->allocate(n, out); }

void mxrt_bm_release(void* h, const int32_t* blocks, int n) { ((BM*)h)->release(blocks, n); }

// match cached full blocks of tokens[0:n]; writes blocks and their 16-byte hashes, returns count
int mxrt_bm_match_prefix(void* h, const int32_t* toks, int n, int32_t* out_blocks, uint64_t* out_hashes) {
    return ((BM*)h)->match_prefix(toks, n, out_blocks, (H128*)out_hashes);
}

// register block (full, tokens toks[0:block_size]) under parent hash; returns the block hash
void mxrt_bm_commit(void* h, int32_t block, const uint64_t* parent, const int32_t* toks, uint64_t* out_hash) {
    H128 p;
    if (parent) {
        p.a = parent[0];
        p.b = parent[1];
    }
    H128 hh = ((BM*)h)->commit(block, p, toks);
    out_hash[0] = hh.a;
    out_hash[1] = hh.b;
}

void mxrt_bm_stats(void* h, int64_t* out) {
    BM* m = (BM*)h;
    out[0] = m->hits;
    out[1] = m->queries;
    out[2] = (int64_t)m->cached.size();
    out[3] = m->num_free();
}

}  // extern "C"
