"""ctypes signatures of libmxrt.so (host runtime: grammar engine, block manager, vector store)."""
import ctypes as C

P, I, I64, U64, F, SZ = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_float, C.c_size_t
CP = C.c_char_p

RT_SIGS = {
    # grammar.cpp
    "mxrt_grammar_parse": (P, [CP, C.c_char_p, I]),
    "mxrt_grammar_free": (None, [P]),
    "mxrt_grammar_num_rules": (I, [P]),
    "mxrt_matcher_new": (P, [P]),
    "mxrt_matcher_clone": (P, [P]),
    "mxrt_matcher_free": (None, [P]),
    "mxrt_matcher_accept": (I, [P, P, I]),
    "mxrt_matcher_is_done": (I, [P]),
    "mxrt_matcher_num_stacks": (I, [P]),
    "mxrt_vocab_new": (P, [P, P, C.c_int32]),
    "mxrt_vocab_free": (None, [P]),
    "mxrt_vocab_num_nodes": (I, [P]),
    "mxrt_matcher_mask": (None, [P, P, P, C.c_int32]),
    "mxrt_matcher_mask_batch": (None, [P, C.c_int, P, P, C.c_int64, C.c_int32, C.c_int]),
    # block_manager.cpp
    "mxrt_bm_new": (P, [I, I, I]),
    "mxrt_bm_free": (None, [P]),
    "mxrt_bm_set_lifo": (None, [P, I]),
    "mxrt_bm_num_free": (I, [P]),
    "mxrt_bm_allocate": (I, [P, I, P]),
    "mxrt_bm_release": (None, [P, P, I]),
    "mxrt_bm_match_prefix": (I, [P, P, I, P, P]),
    "mxrt_bm_commit": (None, [P, C.c_int32, P, P, P]),
    "mxrt_bm_stats": (None, [P, P]),
    # scheduler.cpp
    "mxrt_sched_new": (P, [P, I, I, I, I, I, I]),
    "mxrt_sched_free": (None, [P]),
    "mxrt_sched_table": (P, [P]),
    "mxrt_sched_set_hold": (None, [P, I]),
    "mxrt_sched_add": (I, [P, P, I, I, I]),
    "mxrt_sched_push": (None, [P, I, C.c_int32]),
    "mxrt_sched_pop": (None, [P, I]),
    "mxrt_sched_push_many": (None, [P, P, I]),
    "mxrt_sched_schedule": (I, [P, P]),
    "mxrt_sched_out": (P, [P, I]),
    "mxrt_sched_out_packed": (I, [P, P, I]),
    "mxrt_sched_plan_packed": (I, [P, P, I]),
    "mxrt_sched_add_pending": (None, [P, P, I, I]),
    "mxrt_sched_pending_ok": (I, [P, P, I]),
    "mxrt_sched_plan": (I, [P, P, I, P, I, P]),
    "mxrt_sched_plan_arr": (P, [P, I]),
    "mxrt_sched_commit": (None, [P, P, I]),
    "mxrt_sched_set_prev": (None, [P, P, I]),
    "mxrt_sched_clear_prev": (None, [P]),
    "mxrt_sched_finish": (None, [P, I]),
    "mxrt_sched_abort": (I, [P, I]),
    "mxrt_sched_release_deferred": (I, [P, P]),
    "mxrt_sched_release_slot": (None, [P, I]),
    "mxrt_sched_grow": (I, [P, I, I]),
    "mxrt_sched_blocks": (I, [P, I, P, I]),
    "mxrt_sched_queue": (I, [P, I, P, I]),
    # store.cpp
    "mxrt_store_new": (P, []),
    "mxrt_store_free": (None, [P]),
    "mxrt_store_size": (I64, [P]),
    "mxrt_store_dim": (I, [P]),
    "mxrt_store_set": (I, [P, P, I64, I, P, P]),
    "mxrt_store_delete": (I64, [P, P, I64, I]),
    "mxrt_store_lookup": (None, [P, P, I64, I, P]),
    "mxrt_store_row": (I64, [P, I64, P, P, I64]),
    "mxrt_store_keys_ptr": (P, [P]),
    "mxrt_store_find": (I64, [P, P, I, I64, P, P]),
}


def bind(lib):
    for name, (res, args) in RT_SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
