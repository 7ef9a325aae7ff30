"""DBoW2 TemplatedVocabulary::transform oracle (oracle/orb_bow_oracle.cpp) against an independent
pure-Python reading of Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1260 + BowVector.cpp.
ORBvoc.txt is absent (.MISSING_LARGE_BLOBS), so the vocabularies are synthetic DBoW2-shaped trees
(synth.dbow_vocabulary); parity with the real vocabulary file is unpinned."""
from __future__ import annotations

import math

import numpy as np
import pytest


def python_transform(voc, desc, levelsup):
    cb, ci, vd, wid, wt = voc["child_begin"], voc["child_idx"], voc["desc"], voc["word_id"], voc["weight"]
    L, weighting, scoring = voc["L"], voc.get("weighting", 0), voc.get("scoring", 0)
    tf = weighting in (0, 1)
    must, l1 = scoring != 5, scoring != 1
    bow, fv = {}, {}
    for i, f in enumerate(desc):
        nid_level = L - levelsup
        nid = 0 if nid_level <= 0 else None
        node, level = 0, 0
        while True:
            level += 1
            kids = ci[cb[node]:cb[node + 1]]
            dists = np.unpackbits(np.bitwise_xor(vd[kids], f[None, :]), axis=1).sum(axis=1)
            node = int(kids[int(np.argmin(dists))])  # argmin = first minimum
            if level == nid_level:
                nid = node
            if cb[node + 1] == cb[node]:
                break
        if nid is None:
            nid = node
        w = float(wt[node])
        if w > 0:
            word = int(wid[node])
            if tf:
                bow[word] = bow[word] + w if word in bow else w
            elif word not in bow:
                bow[word] = w
            fv.setdefault(nid, []).append(i)
    if tf and bow and not must:
        nd = float(len(bow))
        bow = {k: v / nd for k, v in bow.items()}
    if must:
        norm = 0.0
        for k in sorted(bow):
            norm += abs(bow[k]) if l1 else bow[k] * bow[k]
        if not l1:
            norm = math.sqrt(norm)
        if norm > 0:
            bow = {k: v / norm for k, v in bow.items()}
    return bow, fv


@pytest.mark.parametrize("k,L,levelsup,weighting,scoring", [(10, 4, 2, 0, 0), (10, 3, 4, 0, 0), (6, 5, 3, 1, 1),
                                                            (8, 4, 1, 2, 0), (10, 4, 2, 3, 5), (5, 4, 2, 0, 5)])
def test_bow_oracle_matches_python(synth, oracle, k, L, levelsup, weighting, scoring):
    voc = synth.dbow_vocabulary(k, L, seed=k * 10 + L, weighting=weighting, scoring=scoring, stop_frac=0.05)
    d = synth.bow_descriptors(voc, 600, seed=L)
    bow, fv = oracle.bow_transform(voc, d, levelsup)
    pbow, pfv = python_transform(voc, d, levelsup)
    assert bow == pbow  # float equality: same operation order
    assert fv == pfv


def test_bow_oracle_edge_cases(synth, oracle):
    voc = synth.dbow_vocabulary(10, 3, seed=3)
    bow, fv = oracle.bow_transform(voc, np.zeros((0, 32), np.uint8), 4)
    assert bow == {} and fv == {}
    # random descriptors (far from every word): ties between children are common
    d = np.random.default_rng(0).integers(0, 256, (500, 32), dtype=np.uint8)
    assert oracle.bow_transform(voc, d, 1) == python_transform(voc, d, 1)
