"""Pure-Python restatement of the reference's MAF readers — TEST INFRASTRUCTURE ONLY.

maf_parser (read_data.py:94-117) and parse_coordinates (read_data.py:150-220) iterate
Biopython's AlignIO MAF records; Biopython is not installed here, so this file restates the
record model of Bio.AlignIO.MafIO the reference relies on ('a' starts a block, a blank line
ends it, 's' lines = src start size strand srcSize text; other lines ignored) and then the
reference's loops verbatim in behaviour.  Parity for MAF ingest is therefore pinned to this
restatement and to hand-written fixtures, not to the reference's own execution.
"""
from itrails_amd.read_data import get_obs_state_dct


def _blocks(path):
    block = []
    with open(path) as f:
        for line in f:
            s = line.strip()
            if not s:
                if block:
                    yield block
                block = []
                continue
            if s.startswith("a") and (len(s) == 1 or s[1].isspace()):
                if block:
                    yield block
                block = []
            elif s.startswith("s") and s[1].isspace():
                f_ = s.split()
                block.append(dict(name=f_[1], start=int(f_[2]), strand=-1 if f_[4] == "-" else 1,
                                  srcSize=int(f_[5]), seq=f_[6]))
    if block:
        yield block


def maf_parser(path, sp_lst):
    order_st = get_obs_state_dct()
    out = []
    for recs in _blocks(path):
        dct = {}
        for r in recs:
            if r["name"].split(".")[0] in sp_lst:
                dct[r["name"].split(".")[0]] = r["seq"].replace("-", "N")
        if len(dct) == 4:
            n = len(recs[-1]["seq"])
            out.append([order_st.index("".join(dct[j][i] for j in sp_lst).upper())
                        for i in range(n)])
    return out


def parse_coordinates(path, sp_lst, ref):
    res = []
    for recs in _blocks(path):
        acc, length, start, strand, size, ref_seq = 0, 0, None, 0, 0, ""
        for r in recs:
            if r["name"].split(".")[0] in sp_lst:
                length = len(r["seq"])
                acc += 1
            if r["name"].split(".")[0] == ref:
                start, strand, size = r["start"], r["strand"], r["srcSize"]
                ref_seq = "".join("1" if c != "-" else "0" for c in r["seq"])
        if acc != 4:
            continue
        if ref_seq == "":
            res.append([-9] * length)
            continue
        st = start if strand == 1 else size - start
        row = []
        for c in ref_seq:
            if c == "1":
                row.append(st)
                st += strand
            else:
                row.append(-9)
        res.append(row)
    return res
