"""Measurement tooling (CPU): the PMC summary's kernel families (tools/pmc_traffic.py) name
each traced kernel as bench.py's roofline expects, so a profile attributes its counters to
the right launch."""
import importlib.util
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def _pmc():
    spec = importlib.util.spec_from_file_location("pmc_traffic", os.path.join(HERE, "..", "tools", "pmc_traffic.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_kernel_families():
    fam = _pmc().family
    ns = "(anonymous namespace)::"
    args = "((anonymous namespace)::DevGraph, (anonymous namespace)::FRec const*)"
    assert fam(f"void {ns}bidi_kernel<16, 9, 128, 64, 7, 1, 0>{args}") == "bidi_kernel<16>"
    assert fam(f"void {ns}bidi_kernel<16, 9, 128, 64, 7, 1, 1>{args}") == "bidi_kernel<16> (pipelined chunks)"
    assert fam(f"{ns}bidi_host_kernel<2>{args}") == "bidi_host_kernel (host batches)"
    assert fam(f"void {ns}bidi_kernel<16, 11, 384, 256, 6, 1, 0>{args}") == "bidi spill stage w (16 requests, 2048 slots)"
    assert fam(f"void {ns}bidi_kernel<1, 13, 1024, 256, 7, 1, 0>{args}") == "bidi single-request stage"
    assert fam(f"void {ns}unit2_kernel<16>{args}") == "unit2_kernel<16>"
    assert fam(f"{ns}part_apply_kernel({ns}PartDev)") == "part_apply_kernel"
    assert fam(f"{ns}part_gather_kernel({ns}PartDev, unsigned long, unsigned long)") == "part_gather_kernel"
    assert fam(f"{ns}clear_kernel(unsigned long*)") is None


def test_label_kernel_families():
    """plan label's kernels and the two-tier label path's (round 5): tier_label_kernel is its
    own family, not label_kernel's"""
    fam = _pmc().family
    ns = "(anonymous namespace)::"
    assert fam(f"void {ns}label_kernel<32, 32>({ns}LabelGraph, unsigned int const*)") == "label_kernel"
    assert fam(f"void {ns}label_full_kernel<32, 32>({ns}LabelGraph)") == "label_full_kernel (overflow lists)"
    assert fam(f"void {ns}label_host_kernel<32, 32>(DevGraph)") == "label_host_kernel (host batches)"
    assert fam(f"void {ns}tier_label_kernel<false>(ketogpu::tier::Graph)") == "tier_label_kernel"
    assert fam(f"{ns}tier_label_reply_kernel(ketogpu::tier::Graph)") == \
        "tier_label exchange kernels (pairs, replies, lengths, bounds)"
    assert fam(f"{ns}tier_pair_kernel(ketogpu::tier::Graph)") == \
        "tier_label exchange kernels (pairs, replies, lengths, bounds)"
    assert fam(f"{ns}tier_reply_len_kernel(ketogpu::tier::Graph)") == "tier_reply kernels (len + scan + copy)"


def test_partitioned_r2_sample_flags_mismatches():
    """bench.py --r2-sample: the independent R2 checker fed from the config #5 row stream agrees
    with the oracle's answers, and a flipped answer is reported"""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(HERE, ".."))
    import bench
    from keto_amd import synth
    from oracle import oracle as O
    w = synth.config5(users=30000, groups=3000, docs=6000, tuples=150000, checks=3000, seed=17)
    st = O.Store(w.namespaces, 100)
    for cols in w.batches(4093):
        st.add_columnar(cols)
    want = st.finalize(presorted=True).check_batch(w.requests(range(w.n_checks)), nthreads=4).astype(bool)
    ok = bench.r2_stream(w, want, 1000)
    assert ok["sample"] == 1000 and ok["mismatches"] == 0
    bad = want.copy()
    bad[:40] ^= True
    assert bench.r2_stream(w, bad, 3000)["mismatches"] == 40
