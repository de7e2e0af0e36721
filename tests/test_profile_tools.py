"""The measurement plumbing (no GPU): bench.py finds the dominant kernel in a rocprof stats map whatever template
arguments the build chose, and tools/pmc_summary.py names the _Float16 k_conv instantiations that rocprofv3 leaves
mangled, so their dispatches are grouped with the other generic layers (profiles/<tag>_pmc.json)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, path))
    mod = importlib.util.module_from_spec(spec)
    saved = sys.argv
    sys.argv = [path]
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.argv = saved
    return mod


def test_bench_finds_the_dominant_kernel_by_pattern():
    bench = _load("bench_under_test", "bench.py")
    stats = {"k_conv_stream<3, 16, 16, 1, true, 4, 0, 4, true>": 0.7,
             "k_conv_stream<5, 16, 16, 1, true, 10, 0, 4, true>": 3.55,
             "k_conv_stream<5, 16, 16, 1, true, 10, 0, 1, false>": 1.2,
             "k_conv<float, 128, true>": 4.6}
    assert bench.kernel_stat(stats, "fp32_split") == ("k_conv_stream<5, 16, 16, 1, true, 10, 0, 4, true>", 3.55)
    assert bench.kernel_stat(stats, "bf16") == ("k_conv_stream<5, 16, 16, 1, true, 10, 0, 1, false>", 1.2)
    assert bench.kernel_stat(stats, "fp32") == ("k_conv<float, 128, true>", 4.6)
    # a build with an extra template argument (e.g. a compute-wave count) still matches
    assert bench.kernel_stat({"k_conv_stream<5, 16, 16, 1, true, 5, 0, 4, true, 8>": 3.1}, "fp32_split")[1] == 3.1
    assert bench.kernel_stat({}, "fp32_split") == (None, None)


def test_pmc_summary_names_mangled_half_instantiations():
    pmc = _load("pmc_summary_under_test", "tools/pmc_summary.py")
    assert pmc.short("_ZN4avse12_GLOBAL__N_16k_convIDF16_Li64ELb1ELb1EEEvNS_8ConvArgsE") == \
        "k_conv<_Float16, 64, true, true>"
    assert pmc.short("_ZN4avse12_GLOBAL__N_16k_convIDF16_Li128ELb0ELb1EEEvNS_8ConvArgsE") == \
        "k_conv<_Float16, 128, false, true>"
    assert pmc.short("void avse::(anonymous namespace)::k_conv_stream<5, 16, 16, 1, true, 10, 0, 4, true>"
                     "(avse::HaloArgs)") == "k_conv_stream<5, 16, 16, 1, true, 10, 0, 4, true>"
    # the generic-layer group takes both spellings
    assert pmc.short("_ZN4avse12_GLOBAL__N_16k_convIDF16_Li64ELb1ELb1EEEvNS_8ConvArgsE").startswith("k_conv<")
