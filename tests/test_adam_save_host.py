"""Host pieces of the ADAM output path (adam_amd/adam_save.py) and of its
test restatement (tests/_adam_ref.py), no device needed: the header lookups
by the device's ids, the run-date parse, the schema (adam.avdl order), and
Java's Float.toString against values whose Java text is documented."""
import pytest

pa = pytest.importorskip("pyarrow")

from _adam_ref import convert_sam, java_float_str  # noqa: E402
from adam_amd import adam_save as A  # noqa: E402


@pytest.mark.parametrize("v,text", [
    (1.0, "1.0"), (100.0, "100.0"), (0.001, "0.001"), (1e-4, "1.0E-4"), (1e7, "1.0E7"), (9999999.0, "9999999.0"),
    (0.1, "0.1"), (1.5, "1.5"), (-2.5, "-2.5"), (0.0, "0.0"), (-0.0, "-0.0"), (3.4028235e38, "3.4028235E38"),
    (123456.7, "123456.7"), (1.0 / 3.0, "0.33333334"), (float("nan"), "NaN"), (float("-inf"), "-Infinity"),
    (12345678.0, "1.2345678E7"),
])
def test_java_float_text(v, text):
    # Float.toString values as the JDK prints them (Float.MAX_VALUE's javadoc: 3.4028235e+38f)
    assert java_float_str(v) == text


def test_header_ids_follow_the_device():
    h = A.HeaderInfo("@HD\tVN:1\n@RG\tID:b\tLB:x\n@RG\tID:a\tPI:300\tDT:2013-06-01T12:30:00Z\n@RG\tID:b\tLB:y\n"
                     "@SQ\tSN:c1\tLN:10\tUR:u\n@SQ\tSN:c2\tLN:20\n")
    # sorted IDs a, b, b: a -> 0, b -> its last index 2 (RecordGroupDictionary's toMap), the last @RG line of b
    assert h.rg_column("ID") == ["a", None, "b"]
    assert h.rg_column("LB") == [None, None, "y"]
    assert h.rg_column("PI", "int") == [300, None, None]
    assert h.rg_column("DT", "date") == [1370089800000, None, None]
    assert h.sq_column("LN", "int") == [10, 20] and h.sq_column("UR") == ["u", None]


@pytest.mark.parametrize("v,ms", [("2013-06-01", 1370044800000), ("2013-06-01T12:30:00+02:00", 1370082600000),
                                  ("2013-06-01T12:30:00.250Z", 1370089800250), ("junk", None)])
def test_run_date(v, ms):
    assert A._iso8601_epoch_ms(v) == ms


def test_schema_is_adam_avdl_order():
    s = A.schema()
    assert s.names[:4] == ["referenceName", "referenceId", "start", "mapq"]
    assert s.names[-4:] == ["referenceLength", "referenceUrl", "mateReferenceLength", "mateReferenceUrl"]
    assert len(s) == 40 and all(f.nullable for f in s)


def test_restatement_attribute_order():
    text = b"@SQ\tSN:c\tLN:9\nq\t0\tc\t1\t60\t1M\t*\t0\t0\tA\tI\tXA:A:c\tNM:i:+1\tAS:i:2\tMD:Z:1\tNM:i:3\n"
    r = convert_sam(text)[0]
    assert r["attributes"] == "AS:i:2\tNM:i:3\tXA:A:c" and r["mismatchingPositions"] == "1"
