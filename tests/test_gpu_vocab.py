"""DBoW2 ORBVocabulary on the GPU vs the CPU oracle (reference Thirdparty/DBoW2/DBoW2/
TemplatedVocabulary.h transform 1126-1256, ScoringObject.cpp L1 score), bit-exact: per-feature
word ids, weights and levelsup nodes; BowVector words and values (double bits); FeatureVector
CSR; L1 scores.  Vocabularies are synthetic trees in the reference's text format
(tests/vocab_cases.py; ORBvoc.txt is not shipped) and the features are real ORB descriptors of
synthetic KITTI-shaped frames plus noisy leaf descriptors.  Also: the vocabulary's FeatureVectors
drive ORBmatcher::SearchByBoW (ORBmatcher.cc:159-288) on the GPU and on the oracle alike."""
import numpy as np
import pytest

import oracle_lib
import search_cases as sc
import vocab_cases as vc

pytestmark = pytest.mark.gpu

VOCABS = {
    "k10L4": dict(k=10, L=4, seed=0),
    "k5L6dfs": dict(k=5, L=6, seed=1, order="dfs"),
    "k8L4_unbalanced_ties": dict(k=8, L=4, seed=2, early_leaf=0.25, dup_children=0.2, trailing_newline=False),
    "k20L3_tf_l2": dict(k=20, L=3, seed=3, scoring=1, weighting=1),
    "k10L3_idf_dot": dict(k=10, L=3, seed=4, scoring=5, weighting=2),
    "k10L3_binary_chi": dict(k=10, L=3, seed=5, scoring=2, weighting=3),
}


@pytest.fixture(scope="module")
def orb_desc():
    (k0, d0), (k1, d1) = sc.frames(0)[0]
    return d0, d1


def _pair(gpu, tmp_path, name):
    p = tmp_path / f"{name}.txt"
    leaves = vc.make_vocab(p, **VOCABS[name])
    g = gpu.ORBVocabulary()
    assert g.loadFromTextFile(p)
    return g, oracle_lib.OracleVocabulary(p), leaves


def _features(leaves, orb_desc, seed):
    return np.concatenate([vc.features_near(leaves, 700, seed=seed), orb_desc[0][:500]])


@pytest.mark.parametrize("name", list(VOCABS))
def test_transform_features_bit_exact(gpu, tmp_path, orb_desc, name):
    g, o, leaves = _pair(gpu, tmp_path, name)
    F = _features(leaves, orb_desc, 7)
    for levelsup in (0, 2, 4, VOCABS[name]["L"] + 1):
        gw, gwt, gn = g.transform_features(F, levelsup)
        ow, owt, on = o.transform_features(F, levelsup)
        assert np.array_equal(gw, ow)
        assert np.array_equal(gwt.view(np.uint64), owt.view(np.uint64))
        assert np.array_equal(gn, on)


@pytest.mark.parametrize("name", list(VOCABS))
def test_transform_bow_and_featvec_bit_exact(gpu, tmp_path, orb_desc, name):
    g, o, leaves = _pair(gpu, tmp_path, name)
    F = _features(leaves, orb_desc, 11)
    bow, fv = g.transform(F, 4)
    bw, bv, fn, fs, ff = o.transform(F, 4)
    assert np.array_equal(bow.words, bw)
    assert np.array_equal(bow.values.view(np.uint64), bv.view(np.uint64))
    assert np.array_equal(fv.node_id, fn) and np.array_equal(fv.start, fs) and np.array_equal(fv.feat, ff)
    assert len(bow) > 100


def test_batch_equals_single_and_edge_sizes(gpu, tmp_path, orb_desc):
    g, o, leaves = _pair(gpu, tmp_path, "k10L4")
    frames = [_features(leaves, orb_desc, s) for s in range(3)]
    frames += [np.zeros((0, 32), np.uint8), orb_desc[1][:1], vc.features_near(leaves, 4096, seed=9)]
    out = g.transform_batch(frames, 4)
    for F, (bow, fv) in zip(frames, out):
        b1, f1 = g.transform(F, 4)
        assert np.array_equal(bow.words, b1.words) and np.array_equal(bow.values, b1.values)
        assert np.array_equal(fv.node_id, f1.node_id) and np.array_equal(fv.feat, f1.feat)
        bw, bv, fn, fs, ff = o.transform(F, 4)
        assert np.array_equal(bow.words, bw) and np.array_equal(bow.values.view(np.uint64), bv.view(np.uint64))
        assert np.array_equal(fv.node_id, fn) and np.array_equal(fv.feat, ff)
    with pytest.raises(gpu.OrbGpuError):
        g.transform(vc.features_near(leaves, 4097, seed=1), 4)


def test_l1_score_bit_exact(gpu, tmp_path, orb_desc):
    g, o, leaves = _pair(gpu, tmp_path, "k10L4")
    vecs = [g.transform(_features(leaves, orb_desc, s), 4)[0] for s in range(12)]
    vecs.append(g.transform(vc.features_near(leaves, 50, seed=99), 4)[0])
    q = vecs[0]
    sc_g = g.score(q, vecs)
    sc_o = np.array([o.score(q.words, q.values, v.words, v.values) for v in vecs])
    assert np.array_equal(sc_g.view(np.uint64), sc_o.view(np.uint64))
    assert sc_g[0] > 0.99 and sc_g[1:].max() < sc_g[0]


def test_empty_vocabulary_clears_outputs(gpu, tmp_path):
    p = tmp_path / "empty.txt"
    p.write_text("10 6  0 0")
    g = gpu.ORBVocabulary()
    assert g.loadFromTextFile(p)
    bow, fv = g.transform(np.zeros((5, 32), np.uint8), 4)
    assert len(bow) == 0 and len(fv.node_id) == 0


def test_vocabulary_featvec_drives_search_by_bow(gpu, tmp_path):
    """Frame::ComputeBoW -> SearchByBoW(pKF, F): the GPU vocabulary's FeatureVectors fed to the GPU
    matcher and the oracle's to the oracle matcher give the same matches."""
    (k0, d0), (k1, d1) = sc.frames(1)[0]
    p = tmp_path / "v.txt"
    # a tree trained on this scene's own descriptors: leaves are the frame's descriptors
    leaves = vc.make_vocab(p, k=10, L=3, seed=4)
    g = gpu.ORBVocabulary()
    assert g.loadFromTextFile(p)
    o = oracle_lib.OracleVocabulary(p)
    _, fv0 = g.transform(d0, 2)
    _, fv1 = g.transform(d1, 2)
    _, _, fn0, fs0, ff0 = o.transform(d0, 2)
    assert np.array_equal(fv0.node_id, fn0) and np.array_equal(fv0.feat, ff0)
    rng = np.random.default_rng(3)
    kf_mp = np.where(rng.random(len(k0)) < 0.8, rng.permutation(len(k0)), -1).astype(np.int32)
    bad = np.zeros(len(k0), np.uint8)
    m = gpu.ORBmatcher(0.75, True)
    n, out = m.SearchByBoW_Frame(d0, k0["angle"], kf_mp, bad, fv0, d1, k1["angle"], fv1)
    on, oout = oracle_lib.oracle_search_by_bow_frame(d0, k0["angle"], kf_mp, bad, fv0, d1, k1["angle"], fv1, 0.75, True)
    assert n == on and np.array_equal(out, oout)
    assert leaves.shape[1] == 32
