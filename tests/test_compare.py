"""`compare -baseqs` (§8 f4, adam_amd/compare.py) on hand-built SAM pairs
with known concordance, and a reference fixture against itself."""
import os

from adam_amd.compare import compare_baseqs, summary

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_resources")

HDR = b"@SQ\tSN:c\tLN:1000\n@RG\tID:g\n"


def _rec(name, flag, qual, rg=b"g"):
    return b"%s\t%d\tc\t10\t60\t%dM\t*\t0\t0\t%s\t%s\tRG:Z:%s\n" % (name, flag, len(qual), b"A" * len(qual), qual, rg)


def test_fixture_against_itself():
    p = os.path.join(GOLD, "artificial.realigned.sam")
    r = compare_baseqs(p, p)
    assert r["count"] > 0 and r["identity"] == r["count"] and r["diff_pct"] == 0.0
    assert r["unique1"] == r["unique2"] == 0
    assert "baseqs" in summary(p, p, r)


def test_known_concordance(tmp_path):
    f1 = HDR + (_rec(b"a", 512, b"IIII") +            # unpaired primary (flag != 0)
                _rec(b"b", 512, b"II") +              # only in file 1
                _rec(b"c", 0x41, b"III") +            # paired, first of pair
                _rec(b"d", 512, b"JJ") + _rec(b"d", 512, b"JJ") +  # two primary reads: size 2, no points
                _rec(b"e", 0, b"KKKK") +              # FLAG 0: unmapped (Q2), no points
                _rec(b"f", 0x101, b"LL"))             # paired, secondary, second of pair
    f2 = HDR + (_rec(b"a", 512, b"IIIH") +
                _rec(b"c", 0x81, b"III") +            # second of pair: another category
                _rec(b"d", 512, b"JJ") + _rec(b"d", 512, b"JJ") +
                _rec(b"e", 0, b"KKKK") +
                _rec(b"f", 0x181, b"LM") +
                _rec(b"z", 512, b"I"))
    p1, p2 = tmp_path / "1.sam", tmp_path / "2.sam"
    p1.write_bytes(f1)
    p2.write_bytes(f2)
    r = compare_baseqs(str(p1), str(p2))
    assert (r["count"], r["identity"]) == (6, 4)       # a: 4 points / 3 equal; f: 2 points / 1 equal
    assert (r["unique1"], r["unique2"]) == (1, 1)       # b, z
    assert abs(r["diff_pct"] - 100.0 * 2 / 6) < 1e-12
    assert r["histogram"][(40, 39)] == 1 and r["histogram"][(43, 44)] == 1


def test_qual_encodings(tmp_path):
    # a char above 0x7F: one latin-1 byte in plain SAM, two UTF-8 bytes in this build's output
    p1, p2 = tmp_path / "1.sam", tmp_path / "2.sam"
    p1.write_bytes(HDR + _rec(b"a", 512, "Ié".encode("latin-1")))
    p2.write_bytes(HDR + _rec(b"a", 512, "Ié".encode("utf-8")).replace(b"2M\t*", b"2M\t*"))
    r = compare_baseqs(str(p1), str(p2), "latin-1", "utf-8")
    assert (r["count"], r["identity"]) == (2, 2)
    assert r["histogram"][((0xE9 - 33) - 256 if 0xE9 - 33 >= 128 else 0xE9 - 33,) * 2] == 1
