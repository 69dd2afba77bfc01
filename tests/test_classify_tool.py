"""CPU checks of tools/classify_graph_race.py, whose output DESIGN.md §5 cites
for the class of round 5's graph wrong-result race.

The classifier regenerates a block of the probe's fill and tests got ^ want
against Z_dist(crc(units i..j)) for every contiguous run of units.  Here it is
fed synthetic records whose answer is known -- a lost tail part, a lost head
part, noise -- and the committed classification of the 60 real records is
re-read.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import classify_graph_race as G  # noqa: E402

import _oracle as O  # noqa: E402


def test_classifier_math_matches_the_oracle():
    data = G.block_bytes(71, 5)
    assert data == O.fill_splitmix(G.MIB, 71, 5 * G.MIB // 8).tobytes()
    assert G.crc(data) == O.crc32(np.frombuffer(data, dtype=np.uint8))
    a, b = data[:300000], data[300000:]
    assert G.crc(data) == G.zshift(G.crc(a), len(b)) ^ G.crc(b)


def test_classifier_finds_a_lost_part():
    seed, block = 73, 9
    data = G.block_bytes(seed, block)
    want = G.crc(data)
    contrib = G.unit_contribs(data, 16384)
    tail = 0
    for k in range(40, 64):  # units 40..63 lost: the tail part
        tail ^= contrib[k]
    r = G.classify(seed, None, block, want ^ tail, want)
    assert r["seed_ok"] and r["class"] == "lost_run"
    assert {"unit": 16384, "units": (40, 63), "of": 64} in r["lost_run"]
    head = 0
    for k in range(0, 7):
        head ^= contrib[k]
    r = G.classify(seed, None, block, want ^ head, want)
    assert r["class"] == "lost_run" and {"unit": 16384, "units": (0, 6), "of": 64} in r["lost_run"]


def test_classifier_reports_noise_as_none():
    seed, block = 74, 3
    want = G.crc(G.block_bytes(seed, block))
    r = G.classify(seed, None, block, want ^ 0x5A5A1234, want)
    assert r["seed_ok"] and r["class"] == "none"


def test_committed_classification_is_all_lost_tail_parts():
    with open(os.path.join(ROOT, "profiles", "r06", "graph_classify", "classes.json")) as f:
        d = json.load(f)
    assert d["classes"] == {"lost_run": 60}
    for e in d["entries"]:
        finest = min(e["lost_run"], key=lambda x: x["unit"])
        i, j = finest["units"]
        assert j == finest["of"] - 1 and i > 0, e  # a tail part: from mid-block to the block end
