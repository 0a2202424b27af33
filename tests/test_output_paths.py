"""Output-path safety of adamSave / transform (host logic, no GPU).

adamSave writes through Hadoop's FileOutputFormat, which refuses an output
path that already exists (FileAlreadyExistsException,
adam-core/.../rdd/AdamRDDFunctions.scala:37-56).  AdamWriter and transform's
sinks do the same; overwrite=True replaces only a regular file or a directory
holding nothing but part files.
"""
import os

import pytest

from adam_amd.adam_save import AdamWriter, is_adam_output


def _part_dir(path):
    os.makedirs(path)
    for name in ("part-r-00000.parquet", "part-r-00001.parquet", "_SUCCESS"):
        open(os.path.join(path, name), "wb").close()


def test_writer_refuses_existing_directory(tmp_path):
    d = tmp_path / "results"
    d.mkdir()
    (d / "keep.txt").write_text("user data")
    with pytest.raises(FileExistsError):
        AdamWriter(str(d))
    with pytest.raises(FileExistsError):  # not a part-file directory: refused even with overwrite
        AdamWriter(str(d), overwrite=True)
    assert (d / "keep.txt").read_text() == "user data"


def test_writer_refuses_existing_output_without_overwrite(tmp_path):
    out = str(tmp_path / "o.adam")
    _part_dir(out)
    with pytest.raises(FileExistsError):
        AdamWriter(out)
    assert is_adam_output(out)


def test_writer_overwrites_part_directory(tmp_path):
    out = str(tmp_path / "o.adam")
    _part_dir(out)
    w = AdamWriter(out, compression="snappy", overwrite=True)
    w.close(True)
    assert sorted(os.listdir(out)) == ["_SUCCESS"]


def test_writer_fresh_path_and_failure_cleanup(tmp_path):
    out = str(tmp_path / "new.adam")
    w = AdamWriter(out, compression="snappy")
    w.close(False)  # a failed job leaves nothing behind
    assert not os.path.exists(out) and not os.path.exists(out + ".partial")
    w = AdamWriter(out, compression="snappy")
    w.close(True)
    assert os.listdir(out) == ["_SUCCESS"]


def test_is_adam_output_rejects_other_content(tmp_path):
    d = tmp_path / "x"
    _part_dir(str(d))
    (d / "notes.md").write_text("x")
    assert not is_adam_output(str(d))
    assert not is_adam_output(str(tmp_path / "missing"))
    f = tmp_path / "file.parquet"
    f.write_bytes(b"PAR1")
    assert not is_adam_output(str(f))


def test_transform_sinks_refuse_directories(tmp_path):
    from adam_amd import transform as T
    d = tmp_path / "dir"
    d.mkdir()
    (d / "keep").write_text("k")
    with pytest.raises(FileExistsError):
        T._SamOut(str(d))
    with pytest.raises(FileExistsError):
        T._SamOut(str(d), overwrite=True)
    with pytest.raises(FileExistsError):
        T._check_out(str(d), True, True)
    assert (d / "keep").read_text() == "k"
    f = tmp_path / "o.sam"
    f.write_text("old")
    with pytest.raises(FileExistsError):
        T._SamOut(str(f))
    s = T._SamOut(str(f), overwrite=True)
    s.close(True)
    assert f.read_bytes() == b""


def test_transform_refuses_before_any_work(tmp_path):
    # the output check comes first: no parse, no device (this runs on CPU)
    from adam_amd import transform as T
    d = tmp_path / "results"
    d.mkdir()
    (d / "keep").write_text("k")
    src = tmp_path / "in.sam"
    src.write_text("@HD\tVN:1.4\n")
    with pytest.raises(FileExistsError):
        T.transform(str(src), str(d), recalibrate=True)
    pq_in = tmp_path / "in.parquet"
    pq_in.write_bytes(b"PAR1")
    with pytest.raises(FileExistsError):
        T.transform(str(pq_in), str(d), recalibrate=True, overwrite=True)
    assert sorted(os.listdir(d)) == ["keep"]
