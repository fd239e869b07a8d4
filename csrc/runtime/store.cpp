// store.cpp — in-memory vector store (the "local-store" backend, N11 of SURVEY §2.3).
//
// Reference semantics (backend/go/stores/store.go): keys are float vectors, values opaque bytes;
// Set merges (an existing key's value is replaced), Delete/Get by exact key, Find returns the
// top-k entries by cosine similarity — with a fast path when every stored key is unit-norm (plain
// dot product). Here keys live in one contiguous row-major float matrix (cache-friendly scans;
// the worker can hand the same matrix to the GPU for very large stores) with an exact-key hash
// index; deletion swaps the last row into the hole (O(1)).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

struct KeyHash {
    size_t operator()(const std::string& s) const { return std::hash<std::string>()(s); }
};

struct Store {
    int dim = -1;
    std::vector<float> keys;      // [n, dim]
    std::vector<float> norms;     // [n]
    std::vector<std::string> vals;
    std::unordered_map<std::string, int64_t, KeyHash> index;  // raw key bytes -> row
    int64_t n_unnormalized = 0;

    int64_t size() const { return (int64_t)vals.size(); }
    static std::string kbytes(const float* k, int dim) { return std::string((const char*)k, dim * sizeof(float)); }
    static bool is_unit(float n) { return std::fabs(n - 1.f) < 1e-4f; }
};

}  // namespace

extern "C" {

void* mxrt_store_new() { return new Store(); }
void mxrt_store_free(void* h) { delete (Store*)h; }
int64_t mxrt_store_size(void* h) { return ((Store*)h)->size(); }
int mxrt_store_dim(void* h) { return ((Store*)h)->dim; }

// keys [n, dim] floats; values concatenated with offsets [n+1]. Returns 0 ok, -1 dim mismatch.
int mxrt_store_set(void* h, const float* keys, int64_t n, int dim, const uint8_t* vals, const int64_t* voff) {
    Store* s = (Store*)h;
    if (s->dim < 0) s->dim = dim;
    if (dim != s->dim) return -1;
    for (int64_t i = 0; i < n; ++i) {
        const float* k = keys + i * dim;
        std::string kb = Store::kbytes(k, dim);
        std::string v((const char*)vals + voff[i], voff[i + 1] - voff[i]);
        auto it = s->index.find(kb);
        if (it != s->index.end()) {
            s->vals[it->second] = std::move(v);
            continue;
        }
        float nn = 0.f;
        for (int d = 0; d < dim; ++d) nn += k[d] * k[d];
        nn = std::sqrt(nn);
        s->index.emplace(std::move(kb), s->size());
        s->keys.insert(s->keys.end(), k, k + dim);
        s->norms.push_back(nn);
        s->vals.push_back(std::move(v));
        if (!Store::is_unit(nn)) s->n_unnormalized++;
    }
    return 0;
}

// delete exact keys; returns number removed
int64_t mxrt_store_delete(void* h, const float* keys, int64_t n, int dim) {
    Store* s = (Store*)h;
    if (dim != s->dim) return 0;
    int64_t removed = 0;
    for (int64_t i = 0; i < n; ++i) {
        auto it = s->index.find(Store::kbytes(keys + i * dim, dim));
        if (it == s->index.end()) continue;
        int64_t row = it->second, last = s->size() - 1;
        if (!Store::is_unit(s->norms[row])) s->n_unnormalized--;
        s->index.erase(it);
        if (row != last) {
            memcpy(&s->keys[row * dim], &s->keys[last * dim], dim * sizeof(float));
            s->norms[row] = s->norms[last];
            s->vals[row] = std::move(s->vals[last]);
            s->index[Store::kbytes(&s->keys[row * dim], dim)] = row;
        }
        s->keys.resize(last * dim);
        s->norms.pop_back();
        s->vals.pop_back();
        ++removed;
    }
    return removed;
}

// get: for each query key, row index or -1
void mxrt_store_lookup(void* h, const float* keys, int64_t n, int dim, int64_t* rows) {
    Store* s = (Store*)h;
    for (int64_t i = 0; i < n; ++i) {
        if (dim != s->dim) { rows[i] = -1; continue; }
        auto it = s->index.find(Store::kbytes(keys + i * dim, dim));
        rows[i] = it == s->index.end() ? -1 : it->second;
    }
}

// read row: key into key_out (dim floats); returns value length, copies up to cap bytes
int64_t mxrt_store_row(void* h, int64_t row, float* key_out, uint8_t* val_out, int64_t cap) {
    Store* s = (Store*)h;
    if (row < 0 || row >= s->size()) return -1;
    if (key_out) memcpy(key_out, &s->keys[row * s->dim], s->dim * sizeof(float));
    const std::string& v = s->vals[row];
    if (val_out) memcpy(val_out, v.data(), std::min<int64_t>(cap, v.size()));
    return (int64_t)v.size();
}

const float* mxrt_store_keys_ptr(void* h) { return ((Store*)h)->keys.data(); }

// top-k by cosine similarity; returns count written (<= k)
int64_t mxrt_store_find(void* h, const float* q, int dim, int64_t k, int64_t* rows, float* sims) {
    Store* s = (Store*)h;
    const int64_t n = s->size();
    if (dim != s->dim || n == 0 || k <= 0) return 0;
    float qn = 0.f;
    for (int d = 0; d < dim; ++d) qn += q[d] * q[d];
    qn = std::sqrt(qn);
    const bool fast = s->n_unnormalized == 0 && Store::is_unit(qn);
    std::vector<std::pair<float, int64_t>> sc(n);
    for (int64_t i = 0; i < n; ++i) {
        const float* kk = &s->keys[i * dim];
        float dot = 0.f;
        for (int d = 0; d < dim; ++d) dot += kk[d] * q[d];
        float sim = fast ? dot : (s->norms[i] > 0 && qn > 0 ? dot / (s->norms[i] * qn) : 0.f);
        sc[i] = {sim, i};
    }
    k = std::min(k, n);
    std::partial_sort(sc.begin(), sc.begin() + k, sc.end(),
                      [](const auto& a, const auto& b) { return a.first > b.first || (a.first == b.first && a.second < b.second); });
    for (int64_t i = 0; i < k; ++i) {
        rows[i] = sc[i].second;
        sims[i] = sc[i].first;
    }
    return k;
}

}  // extern "C"
