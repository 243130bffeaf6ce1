"""Host side of BERT's unpadded rows (vcg_hip.bert.pack_rows): which token rows a TwoStream forward keeps. A padded
position (attention_mask 0) is a masked key of HF BertModel's self-attention (bert_hugface.py:20), so no kept row reads
it, and the pooler reads only position 0 (two_stream.py:178-179): kept = mask != 0, plus position 0, plus every row of
a sequence without any key (HF then attends uniformly over all L positions)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-chapter-generation_amd"))
from vcg_hip.bert import pack_rows  # noqa: E402


def test_prefix_masks():
    m = np.zeros((3, 8), np.int64)
    m[0, :8] = 1
    m[1, :3] = 1
    m[2, :1] = 1
    rows, seq, keys, cls = pack_rows(m)
    assert seq.tolist() == [0, 8, 11, 12]
    assert rows.tolist() == list(range(8)) + [8, 9, 10] + [16]
    assert keys.tolist() == [1] * 12
    assert cls.tolist() == [0, 8, 11]


def test_holes_masked_cls_and_keyless_sequences():
    m = np.zeros((3, 6), np.int64)
    m[0] = [1, 1, 0, 1, 0, 0]   # a hole: positions 0, 1, 3 kept
    m[1] = [0, 0, 1, 1, 0, 0]   # masked CLS: kept anyway (the pooler's row), as a non-key
    # m[2]: no key at all -> every row kept
    rows, seq, keys, cls = pack_rows(m)
    assert seq.tolist() == [0, 3, 6, 12]
    assert rows.tolist() == [0, 1, 3, 6, 8, 9] + list(range(12, 18))
    assert keys.tolist() == [1, 1, 1, 0, 1, 1] + [0] * 6
    assert cls.tolist() == [0, 3, 6]
    assert m.sum() == 5  # (the input is not modified)


def test_random_masks_invariants():
    rng = np.random.default_rng(0)
    m = (rng.random((64, 128)) < 0.7).astype(np.int64)
    m[5] = 0
    rows, seq, keys, cls = pack_rows(m)
    assert np.all(np.diff(rows) > 0) and len(rows) == seq[-1]
    for b in range(64):
        r = rows[seq[b]:seq[b + 1]]
        assert r[0] == b * 128 and np.all(r // 128 == b)  # position 0 first, rows of sequence b only
        want = np.flatnonzero(m[b]) if m[b].any() else np.arange(128)
        assert sorted(set(want.tolist()) | {0}) == (r % 128).tolist()
    assert np.array_equal(keys, m.reshape(-1)[rows])
