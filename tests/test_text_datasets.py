"""paddle.text WMT14 / WMT16 / Conll05st on synthetic archives in the official layouts (no network here: the real
archives cannot be fetched, so the formats are rebuilt from the reference loaders' expectations,
python/paddle/text/datasets/{wmt14,wmt16,conll05}.py)."""
import gzip
import io
import tarfile

import numpy as np
import pytest

from paddle2_amd.text import datasets as D


def _tar(path, members):
    with tarfile.open(path, "w:gz") as tf:
        for name, data in members.items():
            info = tarfile.TarInfo(name)
            info.size = len(data)
            tf.addfile(info, io.BytesIO(data))


def test_wmt14(tmp_path):
    src_dict = "<s>\n<e>\n<unk>\nle\nchat\nnoir\n"
    trg_dict = "<s>\n<e>\n<unk>\nthe\ncat\nblack\n"
    train = "le chat\tthe cat\nle chat noir\tthe black cat\nbad line without tab\n" + \
            ("le " * 80) + "\tthe\n"
    p = tmp_path / "wmt14.tgz"
    _tar(p, {"wmt14/src.dict": src_dict.encode(), "wmt14/trg.dict": trg_dict.encode(),
             "wmt14/train/train": train.encode(), "wmt14/test/test": b"chat inconnu\tcat unknown\n"})
    ds = D.WMT14(str(p), "train", dict_size=5)
    assert len(ds) == 2   # the tab-less line and the >80-id pair are dropped
    src, trg, nxt = ds[1]
    # dict_size 5 keeps ids 0..4: 'noir' (5) and 'black' (5) become <unk> (2)
    np.testing.assert_array_equal(src, [0, 3, 4, 2, 1])
    np.testing.assert_array_equal(trg, [0, 3, 2, 4])
    np.testing.assert_array_equal(nxt, [3, 2, 4, 1])
    te = D.WMT14(str(p), "test", dict_size=10)
    np.testing.assert_array_equal(te[0][0], [0, 4, 2, 1])
    sd, td = ds.get_dict(reverse=True)
    assert sd[4] == "chat" and td[3] == "the"
    with pytest.raises(ValueError):
        D.WMT14(str(p), "train", dict_size=-1)


def test_wmt16_dictionary_by_frequency_and_lang(tmp_path):
    train = "a b b c\tx y\nb c\ty y z\nc\tz\n"
    p = tmp_path / "wmt16.tar.gz"
    _tar(p, {"wmt16/train": train.encode(), "wmt16/test": b"b q\ty\n", "wmt16/val": b"a\tx\n"})
    ds = D.WMT16(str(p), "train", src_dict_size=5, trg_dict_size=6, lang="en")
    en, de = ds.get_dict("en"), ds.get_dict("de")
    assert list(en)[:5] == ["<s>", "<e>", "<unk>", "b", "c"]   # b:3, c:3 (first seen first), a:1 cut
    assert list(de) == ["<s>", "<e>", "<unk>", "y", "z", "x"]
    src, trg, nxt = ds[0]
    np.testing.assert_array_equal(src, [0, 2, 3, 3, 4, 1])
    np.testing.assert_array_equal(trg, [0, 5, 3])
    np.testing.assert_array_equal(nxt, [5, 3, 1])
    te = D.WMT16(str(p), "test", src_dict_size=5, trg_dict_size=6, lang="en")
    np.testing.assert_array_equal(te[0][0], [0, 3, 2, 1])
    de_src = D.WMT16(str(p), "val", src_dict_size=6, trg_dict_size=5, lang="de")   # German source column
    np.testing.assert_array_equal(de_src[0][0], [0, 5, 1])
    assert ds.get_dict("en", reverse=True)[3] == "b"


def test_conll05st(tmp_path):
    # one sentence, two predicates: columns = predicate marks, then one span column per predicate
    words = ["The", "cat", "sat", "on", "mats", ""]
    props = ["-\t(A0*\t*", "-\t*)\t(A0*", "sit\t(V*)\t*)", "-\t(AM-LOC*\t(V*)", "-\t*)\t*", ""]
    props[1] = "-\t*)\t(A0*"
    props[4] = "lie\t*)\t*"
    wz, pz = (gzip.compress(("\n".join(x) + "\n").encode()) for x in (words, props))
    p = tmp_path / "conll05st-tests.tar.gz"
    _tar(p, {"conll05st-release/test.wsj/words/test.wsj.words.gz": wz,
             "conll05st-release/test.wsj/props/test.wsj.props.gz": pz})
    (tmp_path / "w.txt").write_text("<unk>\nThe\ncat\nsat\non\nmats\nbos\neos\n")
    (tmp_path / "v.txt").write_text("sit\nlie\n")
    (tmp_path / "t.txt").write_text("B-A0\nI-A0\nB-V\nI-V\nB-AM-LOC\nI-AM-LOC\nO\n")
    ds = D.Conll05st(str(p), str(tmp_path / "w.txt"), str(tmp_path / "v.txt"), str(tmp_path / "t.txt"))
    assert len(ds) == 2
    assert ds.labels[0] == ["B-A0", "I-A0", "B-V", "B-AM-LOC", "I-AM-LOC"]
    assert ds.labels[1] == ["O", "B-A0", "I-A0", "B-V", "O"]
    wd, vd, ld = ds.get_dict()
    assert list(ld) == ["B-A0", "I-A0", "B-AM-LOC", "I-AM-LOC", "B-V", "I-V", "O"]
    w, n2, n1, c0, p1, p2, pred, mark, lab = ds[0]
    np.testing.assert_array_equal(w, [1, 2, 3, 4, 5])
    assert n2[0] == 1 and n1[0] == 2 and c0[0] == 3 and p1[0] == 4 and p2[0] == 5
    np.testing.assert_array_equal(pred, [0] * 5)
    np.testing.assert_array_equal(mark, [1, 1, 1, 1, 1])
    np.testing.assert_array_equal(lab, [0, 1, 4, 2, 3])
    w, n2, n1, c0, p1, p2, pred, mark, lab = ds[1]   # verb 'on' at index 3: the window runs off the end
    assert c0[0] == 4 and p2[0] == 7 and pred[0] == 1
    np.testing.assert_array_equal(mark, [0, 1, 1, 1, 1])
