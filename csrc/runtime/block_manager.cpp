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
#include <cstdint>
#include <cstring>
#include <deque>
#include <list>
#include <unordered_map>
#include <vector>

namespace {

struct H128 {
    uint64_t a = 0, b = 0;
    bool operator==(const H128& o) const { return a == o.a && b == o.b; }
};
struct H128Hash {
    size_t operator()(const H128& h) const { return h.a ^ (h.b * 0x9E3779B97F4A7C15ull); }
};

H128 hash_block(H128 parent, const int32_t* toks, int n) {
    uint64_t a = 0xcbf29ce484222325ull ^ parent.a, b = 0x84222325cbf29ce4ull ^ parent.b;
    for (int i = 0; i < n; ++i) {
        uint32_t t = (uint32_t)toks[i];
        for (int k = 0; k < 4; ++k) {
            uint8_t x = (t >> (8 * k)) & 0xFF;
            a = (a ^ x) * 0x100000001b3ull;
            b = (b ^ (x + 0x5b)) * 0x100000001b3ull;
        }
    }
    b ^= (uint64_t)n * 0xff51afd7ed558ccdull;
    return {a, b};
}

struct BM {
    int num_blocks, block_size;
    bool prefix;
    std::deque<int32_t> free_list;
    std::vector<int32_t> ref;
    std::vector<H128> hash_of;
    std::vector<uint8_t> has_hash;
    std::vector<std::vector<int32_t>> toks_of;  // verification of cached blocks
    std::unordered_map<H128, int32_t, H128Hash> cached;
    std::list<int32_t> lru;  // evictable (ref == 0, cached)
    std::vector<std::list<int32_t>::iterator> lru_it;
    std::vector<uint8_t> in_lru;
    int64_t hits = 0, queries = 0;

    BM(int nb, int bs, bool pc) : num_blocks(nb), block_size(bs), prefix(pc), ref(nb, 0), hash_of(nb),
                                   has_hash(nb, 0), toks_of(nb), lru_it(nb), in_lru(nb, 0) {
        for (int i = 1; i < nb; ++i) free_list.push_back(i);
    }
    int num_free() const { return (int)free_list.size() + (int)lru.size(); }

    void drop_lru(int32_t b) {
        if (in_lru[b]) {
            lru.erase(lru_it[b]);
            in_lru[b] = 0;
        }
    }
    int32_t take() {
        if (!free_list.empty()) {
            int32_t b = free_list.front();
            free_list.pop_front();
            return b;
        }
        if (!lru.empty()) {
            int32_t b = lru.front();
            lru.pop_front();
            in_lru[b] = 0;
            if (has_hash[b]) {
                auto it = cached.find(hash_of[b]);
                if (it != cached.end() && it->second == b) cached.erase(it);
                has_hash[b] = 0;
                toks_of[b].clear();
            }
            return b;
        }
        return -1;
    }
};

}  // namespace

extern "C" {

void* mxrt_bm_new(int num_blocks, int block_size, int prefix_cache) {
    return new BM(num_blocks, block_size, prefix_cache != 0);
}
void mxrt_bm_free(void* h) { delete (BM*)h; }
int mxrt_bm_num_free(void* h) { return ((BM*)h)->num_free(); }

// allocate n blocks into out; returns 0 on success, -1 if not enough (nothing allocated)
int mxrt_bm_allocate(void* h, int n, int32_t* out) {
    BM* m = (BM*)h;
    if (n > m->num_free()) return -1;
    for (int i = 0; i < n; ++i) {
        int32_t b = m->take();
        m->ref[b] = 1;
        out[i] = b;
    }
    return 0;
}

void mxrt_bm_release(void* h, const int32_t* blocks, int n) {
    BM* m = (BM*)h;
    for (int i = 0; i < n; ++i) {
        int32_t b = blocks[i];
        if (b <= 0 || b >= m->num_blocks) continue;
        if (--m->ref[b] == 0) {
            if (m->has_hash[b] && m->prefix) {
                m->lru.push_back(b);
                m->lru_it[b] = std::prev(m->lru.end());
                m->in_lru[b] = 1;
            } else {
                m->has_hash[b] = 0;
                m->toks_of[b].clear();
                m->free_list.push_back(b);
            }
        }
    }
}

// match cached full blocks of tokens[0:n]; writes blocks and their 16-byte hashes, returns count
int mxrt_bm_match_prefix(void* h, const int32_t* toks, int n, int32_t* out_blocks, uint64_t* out_hashes) {
    BM* m = (BM*)h;
    m->queries++;
    if (!m->prefix || n <= 0) return 0;
    const int bs = m->block_size;
    const int nfull = (n - 1) / bs;
    H128 parent;
    int k = 0;
    for (int i = 0; i < nfull; ++i) {
        H128 hh = hash_block(parent, toks + i * bs, bs);
        auto it = m->cached.find(hh);
        if (it == m->cached.end()) break;
        int32_t b = it->second;
        if (memcmp(m->toks_of[b].data(), toks + i * bs, bs * 4) != 0) break;
        if (m->ref[b] == 0) m->drop_lru(b);
        m->ref[b]++;
        out_blocks[k] = b;
        out_hashes[2 * k] = hh.a;
        out_hashes[2 * k + 1] = hh.b;
        ++k;
        parent = hh;
    }
    if (k) m->hits++;
    return k;
}

// register block (full, tokens toks[0:block_size]) under parent hash; returns the block hash
void mxrt_bm_commit(void* h, int32_t block, const uint64_t* parent, const int32_t* toks, uint64_t* out_hash) {
    BM* m = (BM*)h;
    H128 p;
    if (parent) { p.a = parent[0]; p.b = parent[1]; }
    H128 hh = hash_block(p, toks, m->block_size);
    out_hash[0] = hh.a;
    out_hash[1] = hh.b;
    if (!m->prefix) return;
    if (m->cached.find(hh) == m->cached.end()) {
        m->cached[hh] = block;
        m->hash_of[block] = hh;
        m->has_hash[block] = 1;
        m->toks_of[block].assign(toks, toks + m->block_size);
    }
}

void mxrt_bm_stats(void* h, int64_t* out) {
    BM* m = (BM*)h;
    out[0] = m->hits;
    out[1] = m->queries;
    out[2] = (int64_t)m->cached.size();
    out[3] = m->num_free();
}

}  // extern "C"
