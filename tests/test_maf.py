"""Native MAF reader (itrails_amd/csrc/maf.cpp via itrails_amd.maf) against the Python
restatement of the reference's readers (oracle/maf_oracle.py) on generated MAF files, and
hand-written edge cases.  CPU only."""
import os

import numpy as np
import pytest

from itrails_amd import maf as M
from oracle import maf_oracle as O

SP = ["hg38", "panTro5", "gorGor5", "ponAbe2"]


def _write(path, blocks, header=True):
    with open(path, "w") as f:
        if header:
            f.write("##maf version=1 scoring=none\n# a comment line\n\n")
        for recs in blocks:
            f.write("a score=0.0\n")
            for r in recs:
                if r[0] == "i":
                    f.write(f"i {r[1]} C 0 C 0\n")
                    continue
                name, start, strand, size, seq = r
                f.write(f"s {name} {start} {len(seq) - seq.count('-')} {strand} {size} {seq}\n")
            f.write("\n")


def _random_blocks(rng, nblocks):
    letters = np.array(list("ACTGNactgn-"))
    blocks = []
    for b in range(nblocks):
        L = int(rng.integers(1, 400))
        recs = []
        present = [s for s in SP if rng.random() > 0.08]
        extra = ["rheMac3"] if rng.random() < 0.3 else []
        names = present + extra
        rng.shuffle(names)
        for s in names:
            p = np.array([0.22, 0.22, 0.22, 0.22, 0.01, 0.02, 0.02, 0.02, 0.02, 0.005, 0.02])
            seq = "".join(rng.choice(letters, size=L, p=p / p.sum()))
            recs.append((f"{s}.chr{b % 3 + 1}", int(rng.integers(0, 10**6)),
                         "+" if rng.random() < 0.7 else "-", 10**7, seq))
            if rng.random() < 0.2:
                recs.append(("i", f"{s}.chr1"))
        blocks.append(recs)
    return blocks


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_reader_matches_reference_semantics(tmp_path, seed):
    rng = np.random.default_rng(seed)
    path = tmp_path / "a.maf"
    _write(path, _random_blocks(rng, 60), header=seed != 2)
    ref = O.maf_parser(str(path), SP)
    got = M.maf_parser(str(path), SP)
    assert len(got) == len(ref) > 0
    for g, r in zip(got, ref):
        assert g.dtype == np.int64 and g.tolist() == r
    for refsp in ("hg38", "ponAbe2", "rheMac3"):
        assert M.parse_coordinates(str(path), SP, refsp) == O.parse_coordinates(str(path), SP, refsp)
    obs, off, _, _ = M.read_maf(str(path), SP)
    assert obs.dtype == np.uint16 and off[-1] == len(obs) == sum(len(r) for r in ref)


def test_species_order_and_case(tmp_path):
    path = tmp_path / "b.maf"
    _write(path, [[("ponAbe2.x", 0, "+", 9, "ACgt"), ("hg38.x", 5, "+", 9, "aCTn"),
                   ("gorGor5.x", 0, "-", 9, "G-TA"), ("panTro5.x", 0, "+", 9, "TTTT")]])
    got = M.maf_parser(str(path), SP)
    assert got[0].tolist() == O.maf_parser(str(path), SP)[0]
    # column 0: hg38 A, panTro5 T, gorGor5 G, ponAbe2 A -> "ATGA"
    from itrails_amd.read_data import column_to_index
    assert got[0][0] == column_to_index("ATGA")
    assert got[0][1] == column_to_index("CTNC")  # gap -> N
    assert M.parse_coordinates(str(path), SP, "hg38") == [[5, 6, 7, 8]]
    assert M.parse_coordinates(str(path), SP, "gorGor5") == [[9, -9, 8, 7]]


def test_iupac_code_raises_value_error(tmp_path):
    path = tmp_path / "c.maf"
    _write(path, [[(f"{s}.x", 0, "+", 9, "ACRT") for s in SP]])
    with pytest.raises(ValueError):
        M.maf_parser(str(path), SP)


def test_missing_species_block_dropped_and_empty_file(tmp_path):
    path = tmp_path / "d.maf"
    _write(path, [[(f"{s}.x", 0, "+", 9, "ACGT") for s in SP[:3]],
                  [(f"{s}.x", 0, "+", 9, "AC") for s in SP]])
    assert [g.tolist() for g in M.maf_parser(str(path), SP)] == O.maf_parser(str(path), SP)
    empty = tmp_path / "e.maf"
    empty.write_text("")
    obs, off, _, _ = M.read_maf(str(empty), SP)
    assert len(obs) == 0 and off.tolist() == [0]
    with pytest.raises(FileNotFoundError):
        M.read_maf(str(tmp_path / "missing.maf"), SP)


def test_parallel_scan_equals_sequential(tmp_path, monkeypatch):
    rng = np.random.default_rng(9)
    path = tmp_path / "f.maf"
    _write(path, _random_blocks(rng, 300))
    monkeypatch.setenv("ITR_MAF_THREADS", "1")
    seq = M.read_maf(str(path), SP, "hg38")
    for t in ("3", "7", "64"):
        monkeypatch.setenv("ITR_MAF_THREADS", t)
        par = M.read_maf(str(path), SP, "hg38")
        for a, b in zip(seq, par):
            assert np.array_equal(a, b)
    ref = O.maf_parser(str(path), SP)
    assert [x.tolist() for x in M.maf_parser(str(path), SP)] == ref


def test_duplicate_species_record_block(tmp_path):
    """A block holding two records of one species (hg38.chr1 + hg38.chr5): maf_parser keeps
    it (its dict has 4 keys, read_data.py:106-110) while parse_coordinates drops it (5
    matching records, read_data.py:166-180), exactly like the reference.  The writers then
    see fewer coordinates than decoded columns and must refuse instead of reading past the
    coordinate array."""
    from itrails_amd import writers as W

    path = tmp_path / "dup.maf"
    _write(path, [[(f"{s}.x", 0, "+", 9, "ACGT") for s in SP],
                  [("hg38.chr1", 10, "+", 99, "ACG"), ("hg38.chr5", 20, "+", 99, "TTT")]
                  + [(f"{s}.x", 0, "+", 9, "GGA") for s in SP[1:]]])
    assert [g.tolist() for g in M.maf_parser(str(path), SP)] == O.maf_parser(str(path), SP)
    assert M.parse_coordinates(str(path), SP, "hg38") == O.parse_coordinates(str(path), SP, "hg38")
    obs, off, coords, _ = M.read_maf(str(path), SP, "hg38")
    assert off.tolist() == [0, 4, 7] and len(coords) == 4
    states = np.zeros(len(obs), dtype=np.uint8)
    with pytest.raises(ValueError):
        W.write_viterbi_csv(str(tmp_path / "v.csv"), states, ref_coordinates=coords, block_off=off)
    with pytest.raises(ValueError):
        W.write_posterior_csv(str(tmp_path / "p.csv"), np.full((len(obs), 3), 1 / 3),
                              ref_coordinates=coords, block_off=off)
