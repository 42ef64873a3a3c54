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
