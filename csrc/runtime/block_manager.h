// block_manager.h — paged-KV block allocator with automatic prefix caching, shared by block_manager.cpp (its C
// API) and scheduler.cpp (the native scheduler drives it directly, without a ctypes hop per allocation).
#pragma once
#include <cstdint>
#include <cstring>
#include <deque>
#include <list>
#include <unordered_map>
#include <vector>

namespace mxrt {

struct H128 {
    uint64_t a = 0, b = 0;
    bool operator==(const H128& o) const { return a == o.a && b == o.b; }
};
struct H128Hash {
    size_t operator()(const H128& h) const { return h.a ^ (h.b * 0x9E3779B97F4A7C15ull); }
};

inline H128 hash_block(H128 parent, const int32_t* toks, int n) {
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
    // LIFO reuse: a released block is handed out again first, so the live KV working set stays in a compact range of
    // the pool (fewer distinct pages for the attention kernels' TLBs) instead of drifting through it
    bool lifo = false;

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
    // register a full block (tokens toks[0:block_size]) under its parent's hash; returns the block's hash
    H128 commit(int32_t block, H128 parent, const int32_t* toks) {
        H128 hh = hash_block(parent, toks, block_size);
        if (prefix && cached.find(hh) == cached.end()) {
            cached[hh] = block;
            hash_of[block] = hh;
            has_hash[block] = 1;
            toks_of[block].assign(toks, toks + block_size);
        }
        return hh;
    }
    int allocate(int n, int32_t* out) {
        if (n > num_free()) return -1;
        for (int i = 0; i < n; ++i) {
            int32_t b = take();
            ref[b] = 1;
            out[i] = b;
        }
        return 0;
    }
    void release(const int32_t* blocks, int n) {
        for (int i = 0; i < n; ++i) {
            int32_t b = blocks[i];
            if (b <= 0 || b >= num_blocks) continue;
            if (--ref[b] == 0) {
                if (has_hash[b] && prefix) {
                    lru.push_back(b);
                    lru_it[b] = std::prev(lru.end());
                    in_lru[b] = 1;
                } else {
                    has_hash[b] = 0;
                    toks_of[b].clear();
                    if (lifo) free_list.push_front(b);
                    else free_list.push_back(b);
                }
            }
        }
    }
    // cached full blocks of toks[0:n] (one token is always left to compute); bumps refcounts
    int match_prefix(const int32_t* toks, int n, int32_t* out_blocks, H128* out_hashes) {
        queries++;
        if (!prefix || n <= 0) return 0;
        const int bs = block_size;
        const int nfull = (n - 1) / bs;
        H128 parent;
        int k = 0;
        for (int i = 0; i < nfull; ++i) {
            H128 hh = hash_block(parent, toks + i * bs, bs);
            auto it = cached.find(hh);
            if (it == cached.end()) break;
            int32_t b = it->second;
            if (memcmp(toks_of[b].data(), toks + i * bs, bs * 4) != 0) break;
            if (ref[b] == 0) drop_lru(b);
            ref[b]++;
            out_blocks[k] = b;
            out_hashes[k] = hh;
            ++k;
            parent = hh;
        }
        if (k) hits++;
        return k;
    }
};

}  // namespace mxrt

