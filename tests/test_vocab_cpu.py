"""CPU: the DBoW2 vocabulary oracle pinned by hand-derived known answers, and the product
library's loadFromTextFile (host parse, no GPU) against the oracle's.

Reference: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h (loadFromTextFile 1338-1424, transform
1126-1256), BowVector.cpp, FeatureVector.cpp, ScoringObject.cpp.  No ORBvoc.txt and no DBoW2
test vectors ship with the reference, so the known answers are derived by hand on a k=2, L=2
tree (tests/vocab_cases.tiny_vocab)."""
import numpy as np
import pytest

import oracle_lib
import vocab_cases as vc
import c_orb_slam_amd as orb
from c_orb_slam_amd._lib import ORB_E_INVALID, ORB_E_NODEVICE


def _feat(byte):
    return np.full(32, byte, np.uint8)


def test_tiny_vocabulary_known_answers(tmp_path):
    p = tmp_path / "tiny.txt"
    vc.tiny_vocab(p)
    v = oracle_lib.OracleVocabulary(p)
    assert v.err == 0
    assert v.info() == dict(k=2, L=2, scoring=0, weighting=0, nodes=7, words=4)
    F = np.stack([_feat(b) for b in (0x00, 0x0F, 0xF0, 0xFF, 0xFE, 0xF1)])
    w, wt, nd = v.transform_features(F, levelsup=1)
    # f0 -> a1; f1 ties A/B at 128 (first child A) -> a2; f2 -> A -> a1; f3 -> b2; f4 -> B -> b2; f5 -> b1 (stopped)
    assert w.tolist() == [0, 1, 0, 3, 3, 2]
    assert wt.tolist() == [1.5, 2.0, 1.5, 0.5, 0.5, 0.0]
    assert nd.tolist() == [1, 1, 1, 2, 2, 2]
    bw, bv, fn, fs, ff = v.transform(F, levelsup=1)
    assert bw.tolist() == [0, 1, 3]
    assert bv.tolist() == [3.0 / 6.0, 2.0 / 6.0, 1.0 / 6.0]      # TF-IDF sums, L1-normalised
    assert fn.tolist() == [1, 2] and fs.tolist() == [0, 3, 5] and ff.tolist() == [0, 1, 2, 3, 4]
    # levelsup >= L: the FeatureVector node is the root
    _, _, nd0 = v.transform_features(F, levelsup=2)
    assert (nd0 == 0).all()
    # L1Scoring::score: identical vectors score the rounded sum of 2|v|/2 (1 up to rounding), disjoint 0
    s = 0.0
    for x in bv.tolist():
        s += abs(x - x) - abs(x) - abs(x)
    assert v.score(bw, bv, bw, bv) == -s / 2.0
    assert v.score(bw[:1], [1.0], bw[1:2], [1.0]) == 0.0


def test_trailing_newline_adds_the_stopped_node(tmp_path):
    """saveToTextFile's final endl makes the loader read one more, empty, line (UB in the
    reference; realised as a zero-descriptor, weight-0 leaf under the previous line's parent)."""
    p = tmp_path / "tiny_nl.txt"
    vc.tiny_vocab(p, trailing_newline=True)
    v = oracle_lib.OracleVocabulary(p)
    assert v.info() == dict(k=2, L=2, scoring=0, weighting=0, nodes=8, words=5)


@pytest.mark.parametrize("kw", [dict(k=10, L=4, seed=0), dict(k=5, L=5, seed=1, order="dfs"),
                                dict(k=8, L=4, seed=2, early_leaf=0.2, trailing_newline=False),
                                dict(k=20, L=2, seed=3, scoring=1, weighting=1)])
def test_product_loader_matches_oracle(tmp_path, kw):
    p = tmp_path / "voc.txt"
    vc.make_vocab(p, **kw)
    o = oracle_lib.OracleVocabulary(p)
    g = orb.ORBVocabulary()
    assert g.loadFromTextFile(p)
    assert g.info() == o.info()


def test_loader_rejects_what_the_reference_rejects(tmp_path):
    g = orb.ORBVocabulary()
    assert not g.loadFromTextFile(tmp_path / "missing.txt")
    bad = tmp_path / "bad.txt"
    bad.write_text("21 3  0 0\n")           # m_k > 20 (TemplatedVocabulary.h:1366)
    assert not g.loadFromTextFile(bad)
    assert oracle_lib.OracleVocabulary(bad).err == 2
    assert g.info()["words"] == 0


def test_transform_needs_the_device(tmp_path):
    p = tmp_path / "tiny.txt"
    vc.tiny_vocab(p)
    g = orb.ORBVocabulary()
    assert g.loadFromTextFile(p)
    L = orb.lib()
    assert L.ORBvocabulary_transform(None, None, 0, 4, None) == ORB_E_INVALID
    if not orb.device_available():
        with pytest.raises(orb.OrbGpuError) as ei:
            g.transform(np.zeros((3, 32), np.uint8))
        assert ei.value.code == ORB_E_NODEVICE
