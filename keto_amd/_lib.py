"""ctypes binding of libketogpu.so (include/ketogpu.h).

The library is built in-tree by `python -m keto_amd.build` (or
__graft_entry__.build()).  Loading fails loudly when it is missing: there is no
fallback implementation of any entry point.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KETOGPU_LIB") or os.path.join(HERE, "libketogpu.so")  # override: A/B builds

OK, ENOTFOUND, EINVAL, EDEVICE, ENOMEM, ECOLLISION = 0, 1, 2, 3, 4, 5
SUBJECT_ID, SUBJECT_SET, SUBJECT_NIL = 0, 1, -1
NODE_NONE = 0xFFFFFFFF
NODE_NOT_OWNED = 0xFFFFFFFE
BUILD_SORT = 1
ORDER_NULLS_LAST = 2  # Postgres row order (include/ketogpu.h KETOGPU_ORDER_NULLS_LAST)
ORDERS = {"sqlite": 0, "mysql-bin": 0, "cockroach": 0, "postgres": ORDER_NULLS_LAST}
BUILD_WRITABLE = 4  # rows with free slots: ketogpu_snapshot_write patches in place
WRITE_REASONS = {0: "applied", 1: "not_writable", 2: "wildcard", 3: "poison", 4: "class", 5: "ambiguous",
                 6: "full", 7: "reserve", 8: "fanout"}
NODE_UNION, NODE_LEAF = 0, 1


class KetoError(Exception):
    """A failing libketogpu call; .code is the KETOGPU_E* code."""

    NAMES = {ENOTFOUND: "not_found", EINVAL: "invalid", EDEVICE: "device", ENOMEM: "nomem", ECOLLISION: "collision"}

    def __init__(self, code, msg=""):
        super().__init__(f"{self.NAMES.get(code, code)}: {msg}")
        self.code = code
        self.kind = self.NAMES.get(code, "error")


class Namespace(C.Structure):
    _fields_ = [("id", C.c_int32), ("name", C.c_char_p)]


class RowBatch(C.Structure):
    _fields_ = [
        ("n", C.c_size_t),
        ("namespace_id", C.c_void_p),
        ("object_data", C.c_void_p), ("object_off", C.c_void_p),
        ("relation_data", C.c_void_p), ("relation_off", C.c_void_p),
        ("subject_kind", C.c_void_p),
        ("subject_id_data", C.c_void_p), ("subject_id_off", C.c_void_p),
        ("ss_namespace_id", C.c_void_p),
        ("ss_object_data", C.c_void_p), ("ss_object_off", C.c_void_p),
        ("ss_relation_data", C.c_void_p), ("ss_relation_off", C.c_void_p),
    ]


class BuildOpts(C.Structure):
    _fields_ = [("page_size", C.c_int32), ("flags", C.c_uint32)]


class SnapshotStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "num_rows", "num_bad_rows", "num_groups", "num_nodes", "num_expandable", "num_interior", "num_edges",
        "num_interior_edges", "num_rev_edges", "num_wildcard_nodes", "num_ambiguous_nodes")] + [
        ("build_seconds", C.c_double)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class WriteResult(C.Structure):
    _fields_ = [("applied", C.c_int32), ("reason", C.c_int32)] + [(n, C.c_uint64) for n in (
        "rows_inserted", "rows_deleted", "groups_touched", "device_rows", "new_nodes", "version")] + [
        ("seconds", C.c_double)]

    def as_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_}
        d["applied"] = bool(d["applied"])
        d["reason"] = WRITE_REASONS.get(d["reason"], d["reason"])
        return d


class Subject(C.Structure):
    _fields_ = [("kind", C.c_int32), ("id", C.c_char_p), ("ns", C.c_char_p), ("obj", C.c_char_p),
                ("rel", C.c_char_p)]


class CheckRequest(C.Structure):
    _fields_ = [("ns", C.c_char_p), ("obj", C.c_char_p), ("rel", C.c_char_p), ("subject", Subject)]


class EngineOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("max_words_per_round", C.c_uint32), ("state_budget_bytes", C.c_uint64)]


class RunStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "checks", "rounds", "levels", "frontier_entries", "interior_edges", "rev_edges", "touched", "bytes_push",
        "bytes_pull", "bytes_total")] + [("ms_push", C.c_double), ("ms_pull", C.c_double), ("ms_total", C.c_double)] + [
        ("push_launches", C.c_uint64), ("overflow_retries", C.c_uint64)] + [(n, C.c_uint64) for n in (
        "spilled_units", "unit_rows", "unit_edges", "unit_rev", "bytes_unit")] + [("ms_unit", C.c_double)] + [
        ("spilled_requests", C.c_uint64), ("unit_launches", C.c_uint64), ("main_bytes", C.c_uint64),
        ("main_ms", C.c_double), ("plan", C.c_int32), ("plan_lists", C.c_uint32),
        ("hubs", C.c_uint32), ("hub_words", C.c_uint32), ("hub_build_ms", C.c_double),
        ("plan_unit", C.c_uint32), ("closure_cap_f", C.c_uint32), ("closure_cap_b", C.c_uint32),
        ("closure_nodes_f", C.c_uint64), ("closure_nodes_b", C.c_uint64), ("closure_entries_f", C.c_uint64),
        ("closure_entries_b", C.c_uint64), ("core_build_ms", C.c_double), ("label_on", C.c_int32),
        ("label_coverage", C.c_double), ("label_build_ms", C.c_double), ("label_s_head", C.c_uint32),
        ("label_p_head", C.c_uint32), ("label_pll_ms", C.c_double), ("label_bytes", C.c_uint64),
        ("label_entries", C.c_uint64), ("rest_requests", C.c_uint64), ("full_requests", C.c_uint64),
        ("rest_ms", C.c_double),
        ("label_rewritten", C.c_uint64), ("label_marked", C.c_uint64), ("label_relabels", C.c_uint64)]

    PLANS = {0: "global", 1: "bidi", 2: "v2", 3: "wave", 4: "unit", 5: "lite", 6: "core", 7: "label"}

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class RequestBatch(C.Structure):
    _fields_ = [("n", C.c_size_t)] + [(n, C.c_void_p) for n in (
        "ns_data", "ns_off", "obj_data", "obj_off", "rel_data", "rel_off", "subject_kind", "sid_data", "sid_off",
        "ss_ns_data", "ss_ns_off", "ss_obj_data", "ss_obj_off", "ss_rel_data", "ss_rel_off")]


def request_batch(cols):
    """a RequestBatch over persistence.request_columns() arrays (keep cols alive while used)"""
    ptr = lambda k: cols[k].ctypes.data
    return RequestBatch(cols["n"], ptr("ns_data"), ptr("ns_off"), ptr("obj_data"), ptr("obj_off"), ptr("rel_data"),
                        ptr("rel_off"), ptr("subject_kind"), ptr("sid_data"), ptr("sid_off"), ptr("ss_ns_data"),
                        ptr("ss_ns_off"), ptr("ss_obj_data"), ptr("ss_obj_off"), ptr("ss_rel_data"), ptr("ss_rel_off"))


def row_batch(cols):
    """a RowBatch over persistence.columnar()-style arrays (keep cols alive while used)"""
    ptr = lambda k: None if cols.get(k) is None else cols[k].ctypes.data
    return RowBatch(len(cols["namespace_id"]), ptr("namespace_id"), ptr("object_data"), ptr("object_off"),
                    ptr("relation_data"), ptr("relation_off"), ptr("subject_kind"), ptr("subject_id_data"),
                    ptr("subject_id_off"), ptr("ss_namespace_id"), ptr("ss_object_data"), ptr("ss_object_off"),
                    ptr("ss_relation_data"), ptr("ss_relation_off"))


class GraphView(C.Structure):
    _fields_ = [("num_nodes", C.c_uint32), ("num_expandable", C.c_uint32), ("num_interior", C.c_uint32),
                ("fint_off", C.POINTER(C.c_uint64)), ("fint_col", C.POINTER(C.c_uint32)),
                ("rev_off", C.POINTER(C.c_uint64)), ("rev_col", C.POINTER(C.c_uint32))]


class CoreRecords(C.Structure):
    _fields_ = [("records", C.POINTER(C.c_uint32)), ("num_records", C.c_uint64), ("block_base", C.c_uint64),
                ("block_records", C.c_uint32), ("overflow_rows", C.c_uint64), ("closure_nodes", C.c_uint64),
                ("closure_entries", C.c_uint64)]


class LabelView(C.Structure):
    _fields_ = [("s_head_words", C.c_uint32), ("p_head_words", C.c_uint32),
                ("s_words", C.POINTER(C.c_uint32)), ("p_words", C.POINTER(C.c_uint32)),
                ("num_s_words", C.c_uint64), ("num_p_words", C.c_uint64)] + [(n, C.c_uint64) for n in (
        "s_nodes", "p_nodes", "s_entries", "p_entries", "s_overflow", "p_overflow", "label_entries")] + [
        ("pll_ms", C.c_double), ("build_ms", C.c_double)]


class CommStats(C.Structure):
    _fields_ = [("rccl", C.c_int32), ("loop_self", C.c_int32)] + [(n, C.c_uint64) for n in (
        "sends", "recvs", "allgathers", "allreduces", "bytes_sent")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class TreeNode(C.Structure):
    _fields_ = [("type", C.c_int32), ("num_children", C.c_uint32), ("subject", Subject)]


class Record(C.Structure):
    _fields_ = [("a", C.c_uint32), ("b", C.c_uint32), ("m", C.c_uint64)]


class PartOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("rank", C.c_int32), ("world", C.c_int32), ("record_capacity", C.c_uint64),
                ("max_words_per_round", C.c_uint32), ("state_budget_bytes", C.c_uint64)]


class ShardOpts(C.Structure):
    _fields_ = [("page_size", C.c_int32), ("flags", C.c_uint32), ("rank", C.c_int32), ("world", C.c_int32),
                ("salt", C.c_uint64)]


class ShardStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "rows", "bad_rows", "owned_nodes", "owned_interior", "owned_expandable", "forward_edges",
        "interior_forward_edges", "reverse_edges", "queries", "ambiguous_keys", "num_interior", "num_expandable",
        "num_nodes", "host_bytes")] + [("seconds", C.c_double)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class ShardGraph(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("rank", "world", "num_interior", "num_expandable", "num_nodes",
                                          "owned_interior", "owned_expandable", "owned_nodes")] + [
        ("lf_off", C.POINTER(C.c_uint64)), ("lf_col", C.POINTER(C.c_uint32)),
        ("lr_off", C.POINTER(C.c_uint64)), ("lr_col", C.POINTER(C.c_uint32)),
        ("lb_off", C.POINTER(C.c_uint64)), ("lb_col", C.POINTER(C.c_uint32))]


class PartStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "owned_interior", "owned_expandable", "owned_forward_edges", "owned_reverse_edges", "rounds", "levels",
        "frontier_entries", "forward_edges", "records_sent", "records_received", "queries_answered")] + [
        ("bytes", C.c_uint64 * 8), ("ms", C.c_double * 8), ("launches", C.c_uint64 * 8)]

    KERNELS = ["part_seed_kernel", "part_expand_kernel", "part_count+scatter_kernel", "part_apply_kernel",
               "part_gather_kernel", "part_pull_emit_kernel", "part_pull_answer_kernel", "part_reset_kernel"]

    def as_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_[:11]}
        d["kernels"] = {k: {"bytes": int(self.bytes[i]), "ms": float(self.ms[i]), "launches": int(self.launches[i])}
                        for i, k in enumerate(self.KERNELS)}
        return d


class PartEngineOpts(C.Structure):
    _fields_ = [("direction", C.c_int32), ("record_capacity", C.c_uint64)]


class PartEngineStats(C.Structure):
    _fields_ = [("direction", C.c_int32), ("trial_ns", C.c_uint64 * 2)] + [(n, C.c_uint64) for n in (
        "rounds", "levels", "records_sent", "records_received", "retries", "collectives")] + [
        ("exchange_ms", C.c_double)]

    def as_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_}
        d["trial_ns"] = [int(x) for x in self.trial_ns]
        return d


PART_AUTO = -1
REDUCE_MIN, REDUCE_MAX = 0, 1
COMM_ID_BYTES = 128
# include/ketogpu.h ketogpu_transport callbacks (host memory; 0 = success)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p,
                           C.POINTER(C.c_uint64))
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint32), C.c_uint64, C.c_int32)


class Transport(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("rank", C.c_int32), ("world", C.c_int32), ("allgather", ALLGATHER_FN),
                ("alltoallv", ALLTOALLV_FN), ("allreduce_u32", ALLREDUCE_FN)]


# include/ketogpu.h ketogpu_part_steps callbacks (test hook)
BEGIN_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint64, C.c_int32)
EMIT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64))
APPLY_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64))
STEP_FN = C.CFUNCTYPE(C.c_int, C.c_void_p)
PULL_ANSWER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64)
END_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64))


class PartSteps(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("round_words", C.c_uint64), ("begin", BEGIN_FN), ("emit", EMIT_FN),
                ("apply", APPLY_FN), ("expand", STEP_FN), ("pull_answer", PULL_ANSWER_FN), ("end", END_FN),
                ("abort", STEP_FN)]


# include/ketogpu.h two-tier partitioned mode
class CoreView(C.Structure):
    _fields_ = [("num_interior", C.c_uint32), ("f_off", C.POINTER(C.c_uint64)), ("f_col", C.POINTER(C.c_uint32)),
                ("b_off", C.POINTER(C.c_uint64)), ("b_col", C.POINTER(C.c_uint32)), ("bytes", C.c_uint64)]


class TierOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("max_batch", C.c_uint64), ("fallback_state_bytes", C.c_uint64)]


class TierStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "calls", "batches", "requests", "overflow_requests", "fallback_calls", "queries_sent", "records_sent",
        "records_received", "collectives", "rows_opened", "records_read")] + [
        ("exchange_ms", C.c_double), ("evaluate_ms", C.c_double), ("core_records", C.c_uint64),
        ("seed_records", C.c_uint64), ("eval_kernel_ms", C.c_double), ("eval_kernel_launches", C.c_uint64),
        ("label", C.c_uint64), ("label_words", C.c_uint64), ("label_build_ms", C.c_double)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


TIER_QUERIES_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint64,
                              C.c_void_p, C.POINTER(C.c_uint64))
TIER_REPLY_SIZES_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_uint64))
TIER_REPLY_EMIT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p)
TIER_EVALUATE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint64,
                               C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                               C.POINTER(C.c_uint64))


class TierSteps(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("queries", TIER_QUERIES_FN), ("reply_sizes", TIER_REPLY_SIZES_FN),
                ("reply_emit", TIER_REPLY_EMIT_FN), ("evaluate", TIER_EVALUATE_FN)]


# every symbol declared in include/ketogpu.h, with its ctypes signature
vp, i32, u32, sz = C.c_void_p, C.c_int32, C.c_uint32, C.c_size_t
SIGNATURES = {
    "ketogpu_builder_new": (C.c_int, [C.POINTER(Namespace), sz, C.POINTER(BuildOpts), C.POINTER(vp)]),
    "ketogpu_builder_append": (C.c_int, [vp, C.POINTER(RowBatch)]),
    "ketogpu_builder_finish": (C.c_int, [vp, C.POINTER(vp)]),
    "ketogpu_builder_free": (None, [vp]),
    "ketogpu_snapshot_free": (None, [vp]),
    "ketogpu_snapshot_stats_get": (C.c_int, [vp, C.POINTER(SnapshotStats)]),
    "ketogpu_snapshot_graph": (C.c_int, [vp, C.POINTER(GraphView)]),
    "ketogpu_core_index_build": (C.c_int, [vp, C.POINTER(u32), C.POINTER(u32), C.POINTER(vp)]),
    "ketogpu_core_index_view": (C.c_int, [vp, C.c_int, C.POINTER(CoreRecords)]),
    "ketogpu_core_index_free": (None, [vp]),
    "ketogpu_comm_stats_get": (C.c_int, [vp, C.POINTER(CommStats)]),
    "ketogpu_label_index_build": (C.c_int, [vp, u32, u32, C.POINTER(vp)]),
    "ketogpu_label_index_view": (C.c_int, [vp, C.POINTER(LabelView)]),
    "ketogpu_label_index_free": (None, [vp]),
    "ketogpu_engine_label_heads": (C.c_int, [vp, C.c_int, vp, C.c_uint64, C.POINTER(C.c_uint64),
                                             C.POINTER(C.c_uint32)]),
    "ketogpu_snapshot_save": (C.c_int, [vp, C.c_char_p]),
    "ketogpu_snapshot_apply": (C.c_int, [vp, C.POINTER(RowBatch), C.POINTER(RowBatch), C.POINTER(vp)]),
    "ketogpu_snapshot_load": (C.c_int, [C.c_char_p, C.POINTER(vp)]),
    "ketogpu_snapshot_set_namespaces": (C.c_int, [vp, C.POINTER(Namespace), sz, C.POINTER(vp)]),
    "ketogpu_snapshot_write": (C.c_int, [vp, C.POINTER(RowBatch), C.POINTER(RowBatch), C.POINTER(WriteResult)]),
    "ketogpu_snapshot_version": (C.c_uint64, [vp]),
    "ketogpu_engine_sync": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "ketogpu_engine_check_graph": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
    "ketogpu_resolve": (C.c_int, [vp, C.POINTER(CheckRequest), C.POINTER(u32), C.POINTER(u32)]),
    "ketogpu_resolve_batch": (C.c_int, [vp, C.POINTER(RequestBatch), vp, vp, vp]),
    "ketogpu_engine_new": (C.c_int, [vp, C.POINTER(EngineOpts), C.POINTER(vp)]),
    "ketogpu_engine_free": (None, [vp]),
    "ketogpu_engine_set_events": (C.c_int, [vp, C.c_int]),
    "ketogpu_check": (C.c_int, [vp, C.POINTER(CheckRequest), sz, vp, vp]),
    "ketogpu_check_ids": (C.c_int, [vp, vp, vp, sz, vp, vp]),
    "ketogpu_queries_upload": (C.c_int, [vp, vp, vp, sz, C.POINTER(vp)]),
    "ketogpu_queries_run": (C.c_int, [vp, vp]),
    "ketogpu_queries_run_async": (C.c_int, [vp, vp, C.POINTER(C.c_int)]),
    "ketogpu_engine_wait": (C.c_int, [vp]),
    "ketogpu_probe_random_lines": (C.c_int, [C.c_int, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_double)]),
    "ketogpu_queries_download": (C.c_int, [vp, vp, vp, vp]),
    "ketogpu_queries_free": (None, [vp]),
    "ketogpu_engine_last_stats": (C.c_int, [vp, C.POINTER(RunStats)]),
    "ketogpu_expand": (C.c_int, [vp, C.POINTER(Subject), i32, C.POINTER(vp)]),
    "ketogpu_tree_nodes": (C.c_int, [vp, C.POINTER(C.POINTER(TreeNode)), C.POINTER(sz)]),
    "ketogpu_tree_json": (C.c_int, [vp, C.POINTER(vp)]),
    "ketogpu_tree_free": (None, [vp]),
    "ketogpu_last_error": (C.c_char_p, []),
    "ketogpu_abi_version": (C.c_int, []),
    "ketogpu_free": (None, [vp]),
    "ketogpu_device_count": (C.c_int, []),
    "ketogpu_host_alloc": (C.c_int, [sz, C.POINTER(vp)]),
    "ketogpu_host_free": (None, [vp]),
    "ketogpu_multi_new": (C.c_int, [vp, vp, sz, C.POINTER(EngineOpts), C.POINTER(vp)]),
    "ketogpu_multi_free": (None, [vp]),
    "ketogpu_multi_size": (sz, [vp]),
    "ketogpu_multi_engine": (vp, [vp, sz]),
    "ketogpu_multi_check_ids": (C.c_int, [vp, vp, vp, sz, vp, vp]),
    "ketogpu_multi_range": (None, [sz, sz, sz, C.POINTER(sz), C.POINTER(sz)]),
    "ketogpu_shard_builder_new": (C.c_int, [C.POINTER(Namespace), sz, C.POINTER(ShardOpts), C.POINTER(vp)]),
    "ketogpu_shard_builder_append": (C.c_int, [vp, C.POINTER(RowBatch)]),
    "ketogpu_shard_builder_finish": (C.c_int, [vp, C.POINTER(vp)]),
    "ketogpu_shard_builder_free": (None, [vp]),
    "ketogpu_shard_free": (None, [vp]),
    "ketogpu_shard_counts": (C.c_int, [vp, vp]),
    "ketogpu_shard_set_layout": (C.c_int, [vp, vp]),
    "ketogpu_shard_query_count": (C.c_uint64, [vp]),
    "ketogpu_shard_queries": (C.c_int, [vp, vp, C.c_uint64, vp]),
    "ketogpu_shard_answer": (C.c_int, [vp, vp, C.c_uint64, vp]),
    "ketogpu_shard_apply": (C.c_int, [vp, vp, C.c_uint64]),
    "ketogpu_shard_claim_count": (C.c_uint64, [vp]),
    "ketogpu_shard_claims": (C.c_int, [vp, vp, C.c_uint64, vp]),
    "ketogpu_shard_check_claims": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    "ketogpu_shard_resolve_batch": (C.c_int, [vp, C.POINTER(RequestBatch), vp, vp, vp]),
    "ketogpu_shard_exchange": (C.c_int, [vp, vp]),
    "ketogpu_shard_stats_get": (C.c_int, [vp, C.POINTER(ShardStats)]),
    "ketogpu_shard_view": (C.c_int, [vp, C.POINTER(ShardGraph)]),
    "ketogpu_part_owner": (C.c_uint32, [vp, u32]),
    "ketogpu_part_new": (C.c_int, [vp, C.POINTER(PartOpts), C.POINTER(vp)]),
    "ketogpu_part_free": (None, [vp]),
    "ketogpu_part_round_words": (C.c_uint64, [vp]),
    "ketogpu_part_begin": (C.c_int, [vp, vp, vp, sz]),
    "ketogpu_part_begin_dir": (C.c_int, [vp, vp, vp, sz, C.c_int32]),
    "ketogpu_part_emit": (C.c_int, [vp, vp, C.c_uint64, vp]),
    "ketogpu_part_apply": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    "ketogpu_part_expand": (C.c_int, [vp]),
    "ketogpu_part_pull_emit": (C.c_int, [vp, vp, C.c_uint64, vp]),
    "ketogpu_part_pull_answer": (C.c_int, [vp, vp, C.c_uint64]),
    "ketogpu_part_end": (C.c_int, [vp, vp]),
    "ketogpu_part_abort": (C.c_int, [vp]),
    "ketogpu_part_sync": (C.c_int, [vp]),
    "ketogpu_part_stats_get": (C.c_int, [vp, C.POINTER(PartStats)]),
    "ketogpu_part_set_timing": (C.c_int, [vp, C.c_int32]),
    "ketogpu_comm_unique_id": (C.c_int, [vp]),
    "ketogpu_comm_new": (C.c_int, [vp, C.c_int32, C.c_int32, C.c_int32, C.POINTER(vp)]),
    "ketogpu_comm_from_transport": (C.c_int, [C.POINTER(Transport), C.POINTER(vp)]),
    "ketogpu_comm_free": (None, [vp]),
    "ketogpu_comm_rank": (C.c_int, [vp]),
    "ketogpu_comm_world": (C.c_int, [vp]),
    "ketogpu_part_resolve_batch": (C.c_int, [vp, vp, C.POINTER(RequestBatch), vp, vp, vp]),
    "ketogpu_part_engine_new": (C.c_int, [vp, vp, C.POINTER(PartEngineOpts), C.POINTER(vp)]),
    "ketogpu_part_engine_new_steps": (C.c_int, [C.POINTER(PartSteps), vp, C.POINTER(PartEngineOpts), C.POINTER(vp)]),
    "ketogpu_part_check_ids": (C.c_int, [vp, vp, vp, sz, vp]),
    "ketogpu_part_engine_stats_get": (C.c_int, [vp, C.POINTER(PartEngineStats)]),
    "ketogpu_part_engine_free": (None, [vp]),
    "ketogpu_core_gather": (C.c_int, [vp, vp, C.c_uint64, C.POINTER(vp)]),
    "ketogpu_core_get_view": (C.c_int, [vp, C.POINTER(CoreView)]),
    "ketogpu_core_free": (None, [vp]),
    "ketogpu_tier_new": (C.c_int, [vp, vp, vp, C.POINTER(TierOpts), C.POINTER(vp)]),
    "ketogpu_tier_new_steps": (C.c_int, [C.POINTER(TierSteps), vp, C.POINTER(TierOpts), C.POINTER(vp)]),
    "ketogpu_tier_check_ids": (C.c_int, [vp, vp, vp, sz, vp]),
    "ketogpu_tier_stats_get": (C.c_int, [vp, C.POINTER(TierStats)]),
    "ketogpu_tier_free": (None, [vp]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m keto_amd.build` "
                               "(there is no non-native fallback)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != OK:
        msg = lib().ketogpu_last_error()
        raise KetoError(rc, msg.decode("utf-8", "replace") if msg else "")


def b(s):
    return None if s is None else s.encode("utf-8")
