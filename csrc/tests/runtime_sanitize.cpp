// Host-runtime exerciser for AddressSanitizer / UndefinedBehaviorSanitizer builds (tests/
// test_sanitizers.py compiles csrc/runtime/*.cpp + this file with -fsanitize=address,undefined and
// runs it; no Python in the process, so no sanitizer-runtime preloading is needed).
// Drives the paths the LLM worker hits with untrusted input: GBNF parsing (incl. malformed and
// left-recursive grammars), grammar matching + token masks over a byte vocabulary, the paged-KV block
// manager with the prefix cache (allocate / commit / match / release churn) and the vector store.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

extern "C" {
void* mxrt_grammar_parse(const char* src, char* err, int errlen);
void mxrt_grammar_free(void* h);
void* mxrt_matcher_new(void* gh);
void* mxrt_matcher_clone(void* mh);
void mxrt_matcher_free(void* mh);
int mxrt_matcher_accept(void* mh, const uint8_t* bytes, int n);
int mxrt_matcher_is_done(void* mh);
void* mxrt_vocab_new(const uint8_t* bytes, const int64_t* offsets, int32_t n_tokens);
void mxrt_vocab_free(void* vh);
void mxrt_matcher_mask(void* mh, void* vh, uint32_t* mask, int32_t eos_id);
void* mxrt_bm_new(int num_blocks, int block_size, int prefix_cache);
void mxrt_bm_free(void* h);
int mxrt_bm_num_free(void* h);
int mxrt_bm_allocate(void* h, int n, int32_t* out);
void mxrt_bm_release(void* h, const int32_t* blocks, int n);
int mxrt_bm_match_prefix(void* h, const int32_t* toks, int n, int32_t* out_blocks, uint64_t* out_hashes);
void mxrt_bm_commit(void* h, int32_t block, const uint64_t* parent, const int32_t* toks, uint64_t* out_hash);
void mxrt_bm_stats(void* h, int64_t* out);
void* mxrt_store_new();
void mxrt_store_free(void* h);
int64_t mxrt_store_size(void* h);
int mxrt_store_set(void* h, const float* keys, int64_t n, int dim, const uint8_t* vals, const int64_t* voff);
int64_t mxrt_store_delete(void* h, const float* keys, int64_t n, int dim);
void mxrt_store_lookup(void* h, const float* keys, int64_t n, int dim, int64_t* rows);
int64_t mxrt_store_row(void* h, int64_t row, float* key_out, uint8_t* val_out, int64_t cap);
int64_t mxrt_store_find(void* h, const float* q, int dim, int64_t k, int64_t* rows, float* sims);
}

#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) {                                                        \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                      \
        }                                                                  \
    } while (0)

static int grammars() {
    char err[256];
    const char* bad[] = {"root ::= root \"a\" | \"b\"", "root ::= \"unterminated", "root ::= [a-", "x ::= y",
                         "root ::= (\"a\" | ", "", "root ::= \"\\x\"", "root ::= a\na ::= b\nb ::= a \"c\""};
    for (const char* g : bad) {
        void* h = mxrt_grammar_parse(g, err, sizeof err);
        if (h) mxrt_grammar_free(h);  // some are legal; none may crash or hang
    }
    const char* json_g =
        "root ::= object\n"
        "object ::= \"{\" ws ( string \":\" ws value (\",\" ws string \":\" ws value)* )? \"}\" ws\n"
        "value ::= object | array | string | number | (\"true\" | \"false\" | \"null\") ws\n"
        "array ::= \"[\" ws ( value (\",\" ws value)* )? \"]\" ws\n"
        "string ::= \"\\\"\" ( [^\"\\\\] | \"\\\\\" ([\"\\\\/bfnrt] | \"u\" [0-9a-fA-F]{4}) )* \"\\\"\" ws\n"
        "number ::= (\"-\"? ([0-9] | [1-9] [0-9]*)) (\".\" [0-9]+)? ([eE] [-+]? [0-9]+)? ws\n"
        "ws ::= ([ \\t\\n] ws)?\n";
    void* g = mxrt_grammar_parse(json_g, err, sizeof err);
    CHECK(g != nullptr);
    // byte vocabulary: 256 single bytes + some multi-byte tokens + one empty token
    std::vector<std::string> toks;
    for (int b = 0; b < 256; ++b) toks.push_back(std::string(1, (char)b));
    for (const char* t : {"{\"", "\":", "true", "false", "null", "\xc3\xa9", "\xe2\x82", "12.5e3", ""}) toks.push_back(t);
    std::vector<uint8_t> bytes;
    std::vector<int64_t> off{0};
    for (auto& t : toks) {
        bytes.insert(bytes.end(), t.begin(), t.end());
        off.push_back((int64_t)bytes.size());
    }
    const int n = (int)toks.size();
    void* v = mxrt_vocab_new(bytes.data(), off.data(), n);
    std::vector<uint32_t> mask((n + 31) / 32);
    void* m = mxrt_matcher_new(g);
    const char* doc = "{\"key\": [1, -2.5e3, \"s\\u00e9\", true, {\"n\": null}]}";
    for (const char* p = doc; *p; ++p) {
        mxrt_matcher_mask(m, v, mask.data(), n - 1);
        CHECK(mxrt_matcher_accept(m, (const uint8_t*)p, 1) == 1);
    }
    CHECK(mxrt_matcher_is_done(m) == 1);
    void* c = mxrt_matcher_clone(m);
    CHECK(mxrt_matcher_accept(c, (const uint8_t*)"x", 1) == 0);
    // random byte soup through masks and accepts
    std::mt19937 rng(7);
    void* r = mxrt_matcher_new(g);
    for (int i = 0; i < 2000; ++i) {
        mxrt_matcher_mask(r, v, mask.data(), -1);
        uint8_t b = (uint8_t)(rng() & 0xFF);
        mxrt_matcher_accept(r, &b, 1);
    }
    mxrt_matcher_free(r);
    mxrt_matcher_free(c);
    mxrt_matcher_free(m);
    mxrt_vocab_free(v);
    mxrt_grammar_free(g);
    return 0;
}

static int block_manager() {
    const int NB = 64, BS = 16;
    void* bm = mxrt_bm_new(NB, BS, 1);
    std::mt19937 rng(3);
    std::vector<std::vector<int32_t>> live;
    for (int it = 0; it < 3000; ++it) {
        int n = 1 + (int)(rng() % 6);
        std::vector<int32_t> blocks(n);
        if (rng() % 3 != 0 && mxrt_bm_allocate(bm, n, blocks.data()) == 0) {
            // commit full blocks of a token stream shared by many sequences (prefix cache hits)
            uint64_t parent[2] = {0, 0}, h[2];
            std::vector<int32_t> toks(BS);
            for (int i = 0; i < n; ++i) {
                for (int t = 0; t < BS; ++t) toks[t] = (i * BS + t) % 97 + (int)(rng() % 2);
                mxrt_bm_commit(bm, blocks[i], i ? parent : nullptr, toks.data(), h);
                parent[0] = h[0];
                parent[1] = h[1];
            }
            live.push_back(blocks);
        } else if (!live.empty()) {
            size_t k = rng() % live.size();
            mxrt_bm_release(bm, live[k].data(), (int)live[k].size());
            live.erase(live.begin() + (long)k);
        }
        std::vector<int32_t> q(BS * 5 + 3), ob(8);
        std::vector<uint64_t> oh(16);
        for (size_t t = 0; t < q.size(); ++t) q[t] = (int)(t % 97);
        int k = mxrt_bm_match_prefix(bm, q.data(), (int)q.size(), ob.data(), oh.data());
        CHECK(k >= 0 && k <= 5);
        if (k) mxrt_bm_release(bm, ob.data(), k);
    }
    for (auto& b : live) mxrt_bm_release(bm, b.data(), (int)b.size());
    int32_t junk[3] = {-5, 0, NB + 9};
    mxrt_bm_release(bm, junk, 3);  // out-of-range ids are ignored
    int64_t st[8];
    mxrt_bm_stats(bm, st);
    mxrt_bm_free(bm);
    return 0;
}

static int store() {
    void* s = mxrt_store_new();
    const int D = 8;
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> U(-1, 1);
    for (int round = 0; round < 50; ++round) {
        const int n = 1 + round % 7;
        std::vector<float> keys(n * D);
        for (auto& x : keys) x = U(rng);
        std::vector<uint8_t> vals;
        std::vector<int64_t> voff{0};
        for (int i = 0; i < n; ++i) {
            for (int j = 0; j <= i; ++j) vals.push_back((uint8_t)('a' + j));
            voff.push_back((int64_t)vals.size());
        }
        CHECK(mxrt_store_set(s, keys.data(), n, D, vals.data(), voff.data()) == 0);
        std::vector<int64_t> rows(n);
        mxrt_store_lookup(s, keys.data(), n, D, rows.data());
        std::vector<float> kout(D);
        std::vector<uint8_t> vout(64);
        for (int i = 0; i < n; ++i) CHECK(mxrt_store_row(s, rows[i], kout.data(), vout.data(), 64) == i + 1);
        std::vector<int64_t> fr(4);
        std::vector<float> fs(4);
        mxrt_store_find(s, keys.data(), D, 4, fr.data(), fs.data());
        if (round % 3 == 0) mxrt_store_delete(s, keys.data(), n / 2, D);
    }
    CHECK(mxrt_store_size(s) > 0);
    mxrt_store_free(s);
    return 0;
}

int main() {
    int rc = grammars();
    if (!rc) rc = block_manager();
    if (!rc) rc = store();
    if (!rc) printf("runtime_sanitize: ok\n");
    return rc;
}
