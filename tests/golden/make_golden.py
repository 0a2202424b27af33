#!/usr/bin/env python3
"""Regenerate tests/golden/g1_g2.json: the CPU oracle's outputs for the two
hand-derived golden cases of SURVEY.md Appendix B.

  G1  the ReadCovariatesSuite read (ReadCovariatesSuite.scala:27-35) as the
      whole input: per-base covariates, table, expectedMismatch, apply chars;
  G2  res/artificial.realigned.sam as one partition (the copy under
      tests/golden/reference_resources/): table, expectedMismatch, apply chars.

The fixture is data only (inputs are the committed SAM file / the literal
record below).  tests/test_golden.py checks the oracle against the values
derived by hand from the reference sources and against this fixture; the GPU
parity tests check the HIP path against it.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from adam_amd.records import ADAMRecord, RecordBatch, read_sam  # noqa: E402


def g1_batch():
    r = ADAMRecord(record_group_id=0, read_mapped=True, primary_alignment=True, start=10000, reference_name="1",
                   cigar="10M", mismatching_positions="5C4", sequence="CTACCCTAAC", qual="##LKLPPQ##")
    return RecordBatch.from_records([r])


def g2_batch():
    return read_sam(os.path.join(HERE, "reference_resources", "artificial.realigned.sam"))


def describe(batch, covariates=False):
    d = O.dims_for(batch)
    words, em = O.observe(batch, None, d)
    fin = O.Final(d, words, em)
    out, out_len = O.apply(batch, fin)
    nz = np.nonzero(words)[0]
    res = {
        "dims": [d.n_rg, d.max_len],
        "table_nonzero": {str(int(i)): int(words[i]) for i in nz},
        "expected_mismatch": float(em).hex(),
        "chars": [[int(c) for c in out[int(batch.qual_offset[r]):int(batch.qual_offset[r]) + int(out_len[r])]]
                  for r in range(batch.n_reads)],
    }
    if covariates:
        res["covariates"] = [list(map(int, c)) for c in O.read_covariates(batch, 0)]
    return res


def main():
    fx = {"g1": describe(g1_batch(), covariates=True), "g2": describe(g2_batch())}
    with open(os.path.join(HERE, "g1_g2.json"), "w") as fh:
        json.dump(fx, fh, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "g1_g2.json"))


if __name__ == "__main__":
    main()
