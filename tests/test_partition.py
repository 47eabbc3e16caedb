"""The plan's work placement for the three benchmark layouts, on the host (no GPU).

itr_plan_partition_info runs the host half of itr_plan_create (capi.cpp plan_partition and
the mixed queue) for a given CU count.  Its cost constants (kVitLone, kVitWaveLat, kBulkCu,
kFwdValu, kBulkVit, kVitWaveLatV, kMixFwd, kMixVit) were calibrated at N = 70 on chr10
(DESIGN.md §3.4); these tests pin the decisions they produce, so that a recalibration cannot
move chr10, the chr100 shards or the 100 x 100 kbp layout onto another branch unnoticed.
"""
import numpy as np
import pytest

from itrails_amd import _lib
from itrails_amd.distributed import shard_ranges
from itrails_amd.synth import block_lengths

CUS = 256  # MI355X


def info(lengths, cus=CUS):
    off = np.zeros(len(lengths) + 1, np.int64)
    off[1:] = np.cumsum(lengths)
    out = np.zeros(10, np.int64)
    _lib.check(_lib.lib().itr_plan_partition_info(_lib.ptr(off), len(lengths), cus,
                                                  _lib.ptr(out)))
    keys = ("vit_nlong", "vit_long_cols", "vit_reserve", "fwd_reserve", "wave_ok",
            "vit_nlong_v", "fwd_valu_tasks", "mix_entries", "prune_len", "prune_len_v")
    return dict(zip(keys, out.tolist()))


def geometric(cols):
    # bench.py make_workload: geometric block lengths, mean 2 kbp, seed 12345
    return block_lengths(np.random.default_rng(12345), cols, 2000.0)


@pytest.fixture(scope="module")
def lib():
    try:
        return _lib.lib()
    except ImportError as e:
        pytest.skip(str(e))


def test_chr10(lib):
    """BASELINE config 2 (bench default): 59 long blocks, two at a time per reserved CU on 21
    CUs (one per CU they would need 35: more than 1/8 of the chip), + 14 CUs for the
    forward's VALU halves, also two at a time (one per CU: 20 > kFwdPairMin), in the
    forward+Viterbi call, 69 long blocks in the Viterbi-only call
    (profiles/r4m_vit_long_set.txt: 59..80 long blocks all within 1 % of the best)."""
    d = info(geometric(10_000_000))
    assert d["wave_ok"] == 1
    assert d["vit_nlong"] == 59 and d["vit_reserve"] == 21 and d["fwd_reserve"] == 14
    assert d["vit_nlong_v"] == 69
    assert 40 <= d["vit_nlong"] <= 80 and 59 <= d["vit_nlong_v"] <= 80


def test_chr100_single_gpu(lib):
    """chr100 on one GPU: 50 k blocks, throughput-bound — no long set, per-wave layout, and
    no forward VALU task (every half fits the 70 ms makespan in a matrix-core group: the
    mixed launch takes the whole forward)."""
    d = info(geometric(100_000_000))
    assert d["wave_ok"] == 1
    assert d["vit_nlong"] == 0 and d["vit_nlong_v"] == 0 and d["vit_reserve"] == 0
    assert d["fwd_valu_tasks"] == 0 and d["fwd_reserve"] == 0


@pytest.mark.parametrize("rank", range(8))
def test_chr100_world8_shard(lib, rank):
    """Every shard of the 8-GPU chr100 split keeps the per-wave layout with a long set of
    20-30 blocks (each shard is a chr10-sized alignment)."""
    lengths = geometric(100_000_000)
    lo, hi = shard_ranges(lengths, 8)[rank]
    d = info(lengths[lo:hi])
    assert d["wave_ok"] == 1
    assert 20 <= d["vit_nlong"] <= 30
    assert d["vit_reserve"] + d["fwd_reserve"] <= CUS // 2
    # one long block per reserved CU: the one-per-CU long set is under 1/8 of the chip
    assert d["vit_reserve"] <= CUS // 8
    # the makespan floor of the VALU-task threshold (kMixGroupCol): 6-12 forward CUs, not 20-34
    assert 1 <= d["fwd_reserve"] <= 12
    assert d["vit_nlong_v"] >= d["vit_nlong"]


def test_long_blocks(lib):
    """10 Mbp in 100 blocks of 100 kbp: every block is long, the long work does not fit half
    the chip -> no per-wave layout (the `few` / classic branch of viterbi_impl)."""
    d = info(np.full(100, 100_000, np.int64))
    assert d["wave_ok"] == 0
    assert d["vit_nlong"] == 100 and d["vit_long_cols"] == 10_000_000


@pytest.mark.parametrize("n_blocks", [46, 70, 133])
def test_few_block_sets(lib, n_blocks):
    """The few-block GPU tests (test_gpu_sweeps.py, 5000-column blocks)."""
    d = info(np.full(n_blocks, 5000, np.int64))
    assert d["vit_nlong"] == n_blocks
    assert d["wave_ok"] == (1 if d["vit_reserve"] + d["fwd_reserve"] <= CUS // 2 else 0)


def test_cu_count_scales(lib):
    """Fewer CUs lengthen the bulk makespan, so fewer blocks count as long."""
    lengths = geometric(10_000_000)
    assert info(lengths, 128)["vit_nlong"] <= info(lengths, 256)["vit_nlong"]


def _paired_layout(n_short):
    rng = np.random.default_rng(5)
    return [3000] * 40 + list(rng.integers(100, 600, size=n_short))


def test_long_set_pairing(lib):
    """Two long blocks per reserved CU only when one per CU would take more than 1/8 of the
    chip and the longest fits the makespan at the shared step (capi.cpp kVitPairEff,
    kPairShare): 40 blocks of 3,000 columns beside 2 M columns of short blocks -> 20 CUs;
    the same 40 beside 0.2 M columns (makespan = the longest block's lone sweep) -> 40."""
    assert info(_paired_layout(5600))["vit_reserve"] == 20
    assert info(_paired_layout(600))["vit_reserve"] == 40


def test_prune_lengths(lib):
    """The per-wave Viterbi's bound-pruned step takes the blocks shorter than the expected
    makespan / kPruneCol (1.4 us): chr10's bulk blocks below ~5 kbp (the full scan for the
    longer ones, whose step latency sets the makespan), every block of chr100 on one GPU
    (throughput-bound), ~6.3 kbp in each world-8 shard."""
    d = info(geometric(10_000_000))
    assert 4500 <= d["prune_len"] <= 5500 and 3500 <= d["prune_len_v"] <= 4700
    lengths = geometric(100_000_000)
    assert info(lengths)["prune_len"] > lengths.max()
    for lo, hi in shard_ranges(lengths, 8):
        assert 5500 <= info(lengths[lo:hi])["prune_len"] <= 7000


def test_set_prune_len_rejects_null(lib):
    assert lib.itr_plan_set_prune_len(None, 0) != 0


def test_bad_arguments(lib):
    out = np.zeros(10, np.int64)
    off = np.array([0, 10], np.int64)
    assert lib.itr_plan_partition_info(_lib.ptr(off), 1, 0, _lib.ptr(out)) == _lib.ITR_EINVAL
    bad = np.array([0, 10, 5], np.int64)
    assert lib.itr_plan_partition_info(_lib.ptr(bad), 2, 256, _lib.ptr(out)) == _lib.ITR_EINVAL
