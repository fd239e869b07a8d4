// scheduler.cpp — native continuous-batching scheduler + step planner (the engine's per-step host work that scales
// with the batch: which sequences run, KV block growth / preemption, prefix-cache admission and block hashing, and
// the int32 arrays of the step's forward — tokens, positions, KV slots, logit rows, block tables, prefill offsets,
// overlap fix-up rows).
//
// Same decisions as engine/scheduler.py::Scheduler (kept as the reference implementation and fallback; the
// equivalence is tested step by step in tests/test_native_scheduler.py), in the spirit of the reference's
// update_slots (backend/cpp/llama/grpc-server.cpp:1639-2074) over a paged cache instead of fixed slots.
//
// Per-sequence scalar state lives in ONE int32 table [NF x capacity] that Python maps zero-copy (the engine's
// Sequence objects read / write n_pending etc. through it), token ids / block lists / block hashes in per-slot
// vectors. One call per step builds the whole step; nothing here allocates per token except vector growth.
#include <algorithm>
#include <cstdint>
#include <deque>
#include <vector>

#include "block_manager.h"

namespace {

using mxrt::BM;
using mxrt::H128;

// table fields (rows of the shared int32 table)
enum { F_NC = 0, F_NP, F_ST, F_NCACHED, F_NIDS, F_NPROMPT, F_MAXTOK, F_FLAGS, F_NBLK, F_Q, NF };
enum { ST_WAIT = 0, ST_RUN = 1, ST_FIN = 2 };
enum { Q_NONE = 0, Q_WAIT = 1, Q_RUN = 2, Q_DEF = 3 };
enum { FL_CACHE = 1, FL_HOST = 2, FL_USED = 4 };

struct SSeq {
    std::vector<int32_t> ids;  // prompt + host-known outputs
    std::vector<int32_t> blocks;
    std::vector<H128> hashes;
    int32_t prev_row = -1, prev_gen = 0;
};

struct Sched {
    BM* bm;
    int bs, max_seqs, budget0, max_len, chunk, cap;
    int hold = 0;
    std::vector<int32_t> tab;
    std::vector<SSeq> s;
    std::vector<int32_t> free_slots;
    std::deque<int32_t> waiting;
    std::vector<int32_t> running, deferred;
    std::vector<int32_t> o_dec, o_pf, o_pre;  // o_dec: (slot, start); o_pf: (slot, start, n, sample); o_pre: (slot, failed)
    std::vector<char> drop;
    std::vector<int32_t> dropped;
    int32_t gen = 1;
    int err = 0;
    // plan arrays
    std::vector<int32_t> p[11];
    int32_t meta[6] = {0, 0, 0, 0, 0, 0};

    Sched(BM* m, int bs_, int ms, int mbt, int ml, int pc, int cap_)
        : bm(m), bs(bs_), max_seqs(ms), budget0(mbt), max_len(ml), chunk(pc > 0 ? pc : mbt), cap(cap_),
          tab((size_t)NF * cap_, 0), s(cap_), drop(cap_, 0) {
        free_slots.reserve(cap_);
        for (int i = cap_ - 1; i >= 0; --i) free_slots.push_back(i);
    }

    int32_t& f(int field, int sl) { return tab[(size_t)field * cap + sl]; }
    int total_len(int sl) { return f(F_NIDS, sl) + f(F_NP, sl); }
    bool has_out(int sl) { return f(F_NIDS, sl) > f(F_NPROMPT, sl); }
    int prefill_target(int sl) { return (has_out(sl) || f(F_NP, sl)) ? total_len(sl) - 1 : total_len(sl); }
    bool in_decode(int sl) { return (has_out(sl) || f(F_NP, sl)) && f(F_NC, sl) == total_len(sl) - 1; }
    int blocks_for(int n) { return (n + bs - 1) / bs; }
    int n_generated(int sl) { return f(F_NIDS, sl) - f(F_NPROMPT, sl) + f(F_NP, sl); }

    bool held(int sl) {
        if (!f(F_NP, sl)) return false;
        if (n_generated(sl) >= f(F_MAXTOK, sl) || total_len(sl) >= max_len) return true;
        return hold && (f(F_FLAGS, sl) & FL_HOST);
    }
    void free_blocks(int sl) {
        auto& b = s[sl].blocks;
        if (!b.empty()) {
            bm->release(b.data(), (int)b.size());
            b.clear();
        }
        f(F_NBLK, sl) = 0;
    }
    bool grow(int sl, int ntok) {
        auto& b = s[sl].blocks;
        int need = blocks_for(ntok) - (int)b.size();
        if (need <= 0) return true;
        if (need > bm->num_free()) return false;
        size_t o = b.size();
        b.resize(o + need);
        bm->allocate(need, b.data() + o);
        f(F_NBLK, sl) = (int)b.size();
        return true;
    }
    static void erase(std::vector<int32_t>& v, int32_t x) {
        auto it = std::find(v.begin(), v.end(), x);
        if (it != v.end()) v.erase(it);
    }
    void preempt(int sl) {
        if (f(F_NP, sl)) {  // its in-flight token is not known yet: re-prefill would need it
            err = 1;
            return;
        }
        erase(running, sl);
        free_blocks(sl);
        f(F_NC, sl) = 0;
        s[sl].hashes.clear();
        f(F_ST, sl) = ST_WAIT;
        f(F_Q, sl) = Q_WAIT;
        waiting.push_front(sl);
        o_pre.push_back(sl);
        o_pre.push_back(0);
    }

    int schedule() {
        o_dec.clear();
        o_pf.clear();
        o_pre.clear();
        err = 0;
        int budget = budget0;
        // 1. decode-phase sequences (one token each); grow their block lists, preempting the newest if needed
        std::vector<int32_t> decoding;
        decoding.reserve(running.size());
        for (int32_t sl : running)
            if (in_decode(sl) && !held(sl)) decoding.push_back(sl);
        for (int32_t sl : decoding) {
            if (f(F_Q, sl) != Q_RUN) continue;
            while (!grow(sl, total_len(sl))) {
                int32_t victim = -1;
                for (auto it = running.rbegin(); it != running.rend(); ++it)
                    if (*it != sl && !f(F_NP, *it)) {
                        victim = *it;
                        break;
                    }
                if (victim < 0) break;
                preempt(victim);
                if (err) return -1;
                drop[victim] = 1;
                dropped.push_back(victim);
            }
            if (f(F_Q, sl) != Q_RUN) continue;
            if (blocks_for(total_len(sl)) > (int)s[sl].blocks.size()) {
                if (!f(F_NP, sl)) preempt(sl);  // could not grow even after preemption (with a token in flight: sit out)
                drop[sl] = 1;
                dropped.push_back(sl);
            }
        }
        for (int32_t sl : decoding) {
            if (drop[sl]) continue;
            o_dec.push_back(sl);
            o_dec.push_back(f(F_NC, sl));
        }
        for (int32_t sl : dropped) drop[sl] = 0;
        dropped.clear();
        budget -= (int)o_dec.size() / 2;
        // 2. continuing prefills of running sequences (chunked)
        for (int32_t sl : running) {
            if (in_decode(sl) || budget <= 0) continue;
            int n = std::min({prefill_target(sl) - f(F_NC, sl), budget, chunk});
            if (n <= 0 || !grow(sl, f(F_NC, sl) + n)) continue;
            bool done = f(F_NC, sl) + n >= prefill_target(sl);
            o_pf.insert(o_pf.end(), {sl, f(F_NC, sl), n, (int32_t)(done && !has_out(sl) && !f(F_NP, sl))});
            budget -= n;
        }
        // 3. admit new sequences (FIFO), reusing cached prefix blocks first
        while (!waiting.empty() && budget > 0 && (int)running.size() < max_seqs) {
            int32_t sl = waiting.front();
            SSeq& q = s[sl];
            if (q.blocks.empty() && f(F_NC, sl) == 0) {
                int k = 0;
                if (f(F_FLAGS, sl) & FL_CACHE) {
                    int n = prefill_target(sl);
                    int capb = std::max(1, (n - 1) / bs);
                    q.blocks.resize(capb);
                    q.hashes.resize(capb);
                    k = bm->match_prefix(q.ids.data(), n, q.blocks.data(), q.hashes.data());
                }
                q.blocks.resize(k);
                q.hashes.resize(k);
                f(F_NBLK, sl) = k;
                f(F_NC, sl) = k * bs;
                f(F_NCACHED, sl) = k * bs;
            }
            int n = std::min({prefill_target(sl) - f(F_NC, sl), budget, chunk});
            if (!grow(sl, f(F_NC, sl) + n)) {
                if (running.empty()) {  // nothing can free memory: fail this request rather than deadlock
                    waiting.pop_front();
                    free_blocks(sl);
                    f(F_ST, sl) = ST_FIN;
                    f(F_Q, sl) = Q_NONE;
                    o_pre.push_back(sl);
                    o_pre.push_back(1);
                    continue;
                }
                break;
            }
            waiting.pop_front();
            f(F_ST, sl) = ST_RUN;
            f(F_Q, sl) = Q_RUN;
            running.push_back(sl);
            bool done = f(F_NC, sl) + n >= prefill_target(sl);
            o_pf.insert(o_pf.end(), {sl, f(F_NC, sl), n, (int32_t)(done && !has_out(sl))});
            budget -= n;
        }
        return 0;
    }

    // arrays of one forward step (engine._plan): decode rows first, then the prefill chunks
    int plan(const int32_t* dec, int nd, const int32_t* pf, int npf) {
        int T = nd;
        for (int k = 0; k < npf; ++k) T += pf[4 * k + 2];
        for (auto& a : p) a.clear();
        auto &tok = p[0], &pos = p[1], &slot = p[2], &lidx = p[3], &dbt = p[4], &dlen = p[5], &pbt = p[6],
             &pcu = p[7], &pctx = p[8], &fdst = p[9], &fsrc = p[10];
        tok.resize(T);
        pos.resize(T);
        slot.resize(T);
        int i = 0, dmaxb = 0, pmaxb = 0;
        for (int k = 0; k < nd; ++k, ++i) {
            int sl = dec[k];
            SSeq& q = s[sl];
            int ps = f(F_NC, sl);
            if (f(F_NP, sl)) {  // input sampled by the previous, still unread step: gathered on the device
                if (q.prev_gen != gen) return -2;
                tok[i] = 0;
                fdst.push_back(i);
                fsrc.push_back(q.prev_row);
            } else {
                tok[i] = q.ids.back();
            }
            pos[i] = ps;
            slot[i] = q.blocks[ps / bs] * bs + ps % bs;
            dmaxb = std::max(dmaxb, (int)q.blocks.size());
        }
        for (int k = 0; k < npf; ++k) {
            int sl = pf[4 * k], st = pf[4 * k + 1], n = pf[4 * k + 2];
            SSeq& q = s[sl];
            if (st + n > (int)q.ids.size()) return -3;  // prompt rows must be host-known
            for (int r = 0; r < n; ++r, ++i) {
                int ps = st + r;
                tok[i] = q.ids[ps];
                pos[i] = ps;
                slot[i] = q.blocks[ps / bs] * bs + ps % bs;
            }
            pmaxb = std::max(pmaxb, (int)q.blocks.size());
        }
        for (int k = 0; k < nd; ++k) lidx.push_back(k);
        int off = nd;
        for (int k = 0; k < npf; ++k) {
            if (pf[4 * k + 3]) lidx.push_back(off + pf[4 * k + 2] - 1);
            off += pf[4 * k + 2];
        }
        if (nd) {
            dbt.assign((size_t)nd * dmaxb, 0);
            dlen.resize(nd);
            for (int k = 0; k < nd; ++k) {
                const auto& b = s[dec[k]].blocks;
                std::copy(b.begin(), b.end(), dbt.begin() + (size_t)k * dmaxb);
                dlen[k] = f(F_NC, dec[k]) + 1;
            }
        }
        if (npf) {
            pbt.assign((size_t)npf * pmaxb, 0);
            pcu.assign(npf + 1, 0);
            pctx.resize(npf);
            for (int k = 0; k < npf; ++k) {
                const auto& b = s[pf[4 * k]].blocks;
                std::copy(b.begin(), b.end(), pbt.begin() + (size_t)k * pmaxb);
                pcu[k + 1] = pcu[k] + pf[4 * k + 2];
                pctx[k] = pf[4 * k + 1] + pf[4 * k + 2];
            }
        }
        meta[0] = T;
        meta[1] = (int)lidx.size();
        meta[2] = dmaxb;
        meta[3] = pmaxb;
        meta[4] = (int)fdst.size();
        return 0;
    }

    // KV bookkeeping after the forward: computed lengths, and newly full blocks into the prefix cache
    void commit_one(int sl, int start, int n) {
        f(F_NC, sl) = start + n;
        if (!(f(F_FLAGS, sl) & FL_CACHE)) return;  // e.g. image placeholders: token ids do not identify the KV
        SSeq& q = s[sl];
        int nfull = std::min(f(F_NC, sl), f(F_NIDS, sl)) / bs;  // only blocks whose ids are all host-known
        while ((int)q.hashes.size() < nfull) {
            size_t i = q.hashes.size();
            H128 parent = i ? q.hashes[i - 1] : H128{};
            q.hashes.push_back(bm->commit(q.blocks[i], parent, q.ids.data() + i * bs));
        }
    }

    void finish(int sl) {
        f(F_ST, sl) = ST_FIN;
        if (f(F_Q, sl) == Q_RUN) erase(running, sl);
        if (f(F_Q, sl) == Q_WAIT) {
            auto it = std::find(waiting.begin(), waiting.end(), sl);
            if (it != waiting.end()) waiting.erase(it);
        }
        if (f(F_Q, sl) == Q_DEF) return;
        if (f(F_NP, sl)) {  // a launched step still writes its KV blocks
            deferred.push_back(sl);
            f(F_Q, sl) = Q_DEF;
        } else {
            free_blocks(sl);
            f(F_Q, sl) = Q_NONE;
        }
    }

    int abort(int sl) {
        int q = f(F_Q, sl);
        if (q == Q_RUN) {
            erase(running, sl);
        } else if (q == Q_WAIT) {
            auto it = std::find(waiting.begin(), waiting.end(), sl);
            if (it != waiting.end()) waiting.erase(it);
        } else {
            return 0;
        }
        if (f(F_NP, sl)) {
            deferred.push_back(sl);
            f(F_Q, sl) = Q_DEF;
        } else {
            free_blocks(sl);
            f(F_Q, sl) = Q_NONE;
        }
        return 1;
    }
};

}  // namespace

extern "C" {

void* mxrt_sched_new(void* bm, int block_size, int max_num_seqs, int max_batched_tokens, int max_model_len,
                     int prefill_chunk, int capacity) {
    return new Sched((BM*)bm, block_size, max_num_seqs, max_batched_tokens, max_model_len, prefill_chunk, capacity);
}
void mxrt_sched_free(void* h) { delete (Sched*)h; }
int32_t* mxrt_sched_table(void* h) { return ((Sched*)h)->tab.data(); }
void mxrt_sched_set_hold(void* h, int hold) { ((Sched*)h)->hold = hold; }

// a new sequence (WAITING, queued FIFO); flags: 1 cache_prompt, 2 needs host state. Returns its slot, -1 when full.
int mxrt_sched_add(void* h, const int32_t* prompt, int n, int max_tokens, int flags) {
    Sched* m = (Sched*)h;
    if (m->free_slots.empty()) return -1;
    int sl = m->free_slots.back();
    m->free_slots.pop_back();
    SSeq& q = m->s[sl];
    q.ids.assign(prompt, prompt + n);
    q.blocks.clear();
    q.hashes.clear();
    q.prev_gen = 0;
    for (int k = 0; k < NF; ++k) m->f(k, sl) = 0;
    m->f(F_NIDS, sl) = n;
    m->f(F_NPROMPT, sl) = n;
    m->f(F_MAXTOK, sl) = max_tokens;
    m->f(F_FLAGS, sl) = flags | FL_USED;
    m->f(F_ST, sl) = ST_WAIT;
    m->f(F_Q, sl) = Q_WAIT;
    m->waiting.push_back(sl);
    return sl;
}

// host-known output tokens (appended after their step was read) / the EOS that is dropped from the output
void mxrt_sched_push(void* h, int sl, int32_t tok) {
    Sched* m = (Sched*)h;
    m->s[sl].ids.push_back(tok);
    m->f(F_NIDS, sl) = (int)m->s[sl].ids.size();
}
void mxrt_sched_pop(void* h, int sl) {
    Sched* m = (Sched*)h;
    auto& ids = m->s[sl].ids;
    if ((int)ids.size() > m->f(F_NPROMPT, sl)) ids.pop_back();
    m->f(F_NIDS, sl) = (int)ids.size();
}

// batched form of push / pop: (slot, token) pairs in order; token < 0 pops
void mxrt_sched_push_many(void* h, const int32_t* pairs, int n) {
    for (int k = 0; k < n; ++k) {
        if (pairs[2 * k + 1] >= 0)
            mxrt_sched_push(h, pairs[2 * k], pairs[2 * k + 1]);
        else
            mxrt_sched_pop(h, pairs[2 * k]);
    }
}

// one step's schedule; counts = (decode rows, prefill chunks, preempted). 0, or -1 (preempting a sequence with a
// token in flight: a caller bug)
int mxrt_sched_schedule(void* h, int32_t* counts) {
    Sched* m = (Sched*)h;
    int rc = m->schedule();
    counts[0] = (int)m->o_dec.size() / 2;
    counts[1] = (int)m->o_pf.size() / 4;
    counts[2] = (int)m->o_pre.size() / 2;
    return rc;
}
// the last schedule's outputs packed into out: dec (slot, start) pairs, pf quads, preempted pairs; returns ints written
int mxrt_sched_out_packed(void* h, int32_t* out, int cap) {
    Sched* m = (Sched*)h;
    size_t n = m->o_dec.size() + m->o_pf.size() + m->o_pre.size();
    if ((int)n > cap) return -1;
    out = std::copy(m->o_dec.begin(), m->o_dec.end(), out);
    out = std::copy(m->o_pf.begin(), m->o_pf.end(), out);
    std::copy(m->o_pre.begin(), m->o_pre.end(), out);
    return (int)n;
}

// the last plan's arrays concatenated in index order 0..10 (sizes: meta of mxrt_sched_plan); returns ints written
int mxrt_sched_plan_packed(void* h, int32_t* out, int cap) {
    Sched* m = (Sched*)h;
    size_t n = 0;
    for (auto& a : m->p) n += a.size();
    if ((int)n > cap) return -1;
    for (auto& a : m->p) out = std::copy(a.begin(), a.end(), out);
    return (int)n;
}

// every decode slot with a token in flight finds it in the last launched step (engine._pending_on_device)
int mxrt_sched_pending_ok(void* h, const int32_t* slots, int n) {
    Sched* m = (Sched*)h;
    for (int k = 0; k < n; ++k) {
        const int sl = slots[k];
        if (m->f(F_NP, sl) && m->s[sl].prev_gen != m->gen) return 0;
    }
    return 1;
}

// n_pending += d for each slot (a launched step's sampled rows: +1; their read-back: -1)
void mxrt_sched_add_pending(void* h, const int32_t* slots, int n, int d) {
    Sched* m = (Sched*)h;
    for (int k = 0; k < n; ++k) m->f(F_NP, slots[k]) += d;
}

const int32_t* mxrt_sched_out(void* h, int which) {
    Sched* m = (Sched*)h;
    return which == 0 ? m->o_dec.data() : which == 1 ? m->o_pf.data() : m->o_pre.data();
}

// plan arrays of (dec slots, pf (slot, start, n, sample) entries); meta = (T, logit rows, dec max blocks, pf max
// blocks, fix rows). 0, -2 (a pending input whose previous step is not the current one), -3 (prompt rows unknown)
int mxrt_sched_plan(void* h, const int32_t* dec, int nd, const int32_t* pf, int npf, int32_t* meta) {
    Sched* m = (Sched*)h;
    int rc = m->plan(dec, nd, pf, npf);
    for (int k = 0; k < 5; ++k) meta[k] = m->meta[k];
    return rc;
}
// 0 tokens 1 positions 2 slots 3 lidx 4 dec_bt 5 dec_lens 6 pf_bt 7 pf_cu 8 pf_ctx 9 fix_dst 10 fix_src
const int32_t* mxrt_sched_plan_arr(void* h, int which) { return ((Sched*)h)->p[which].data(); }

// items: (slot, start, n) triples of the step's decode rows and prefill chunks
void mxrt_sched_commit(void* h, const int32_t* items, int n) {
    Sched* m = (Sched*)h;
    for (int k = 0; k < n; ++k) m->commit_one(items[3 * k], items[3 * k + 1], items[3 * k + 2]);
}

// the rows of the last launched sampling step (decode inputs still in flight are gathered from them)
void mxrt_sched_set_prev(void* h, const int32_t* slots, int n) {
    Sched* m = (Sched*)h;
    ++m->gen;
    for (int k = 0; k < n; ++k) {
        m->s[slots[k]].prev_row = k;
        m->s[slots[k]].prev_gen = m->gen;
    }
}
void mxrt_sched_clear_prev(void* h) { ++((Sched*)h)->gen; }

void mxrt_sched_finish(void* h, int sl) { ((Sched*)h)->finish(sl); }
int mxrt_sched_abort(void* h, int sl) { return ((Sched*)h)->abort(sl); }

// free the blocks of deferred (finished) sequences whose in-flight steps were all read; returns them in out
int mxrt_sched_release_deferred(void* h, int32_t* out) {
    Sched* m = (Sched*)h;
    int n = 0;
    std::vector<int32_t> keep;
    for (int32_t sl : m->deferred) {
        if (m->f(F_NP, sl)) {
            keep.push_back(sl);
        } else {
            m->free_blocks(sl);
            m->f(F_Q, sl) = Q_NONE;
            out[n++] = sl;
        }
    }
    m->deferred.swap(keep);
    return n;
}

// the slot's sequence is gone from every queue: recycle it (frees blocks it still holds)
void mxrt_sched_release_slot(void* h, int sl) {
    Sched* m = (Sched*)h;
    if (!(m->f(F_FLAGS, sl) & FL_USED)) return;
    m->abort(sl);
    if (m->f(F_Q, sl) == Q_DEF) Sched::erase(m->deferred, sl);
    m->free_blocks(sl);
    m->f(F_FLAGS, sl) = 0;
    m->f(F_Q, sl) = Q_NONE;
    std::vector<int32_t>().swap(m->s[sl].ids);
    std::vector<H128>().swap(m->s[sl].hashes);
    m->free_slots.push_back(sl);
}

int mxrt_sched_grow(void* h, int sl, int ntok) { return ((Sched*)h)->grow(sl, ntok) ? 1 : 0; }

int mxrt_sched_blocks(void* h, int sl, int32_t* out, int cap) {
    Sched* m = (Sched*)h;
    const auto& b = m->s[sl].blocks;
    int n = std::min(cap, (int)b.size());
    std::copy(b.begin(), b.begin() + n, out);
    return (int)b.size();
}

// which: 0 waiting (FIFO order), 1 running, 2 deferred; returns the count (writes at most cap)
int mxrt_sched_queue(void* h, int which, int32_t* out, int cap) {
    Sched* m = (Sched*)h;
    int n = 0;
    if (which == 0) {
        for (int32_t sl : m->waiting)
            if (n < cap) out[n++] = sl;
        return (int)m->waiting.size();
    }
    const auto& v = which == 1 ? m->running : m->deferred;
    for (int32_t sl : v)
        if (n < cap) out[n++] = sl;
    return (int)v.size();
}

}  // extern "C"
