"""N1 dataset_reader (staytime/parse.py:73-92): TFRecord framing with CRC32C, tf.train.Example
decoding with parse.py:17-23's spec, file listing, per-worker sharding, interleave, batching; the
device half (parse_input_func labels) in the -m gpu test."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from recommendsystem_amd import data as D

SLOTS = ["1568", "1570", "2125"]


def _examples(rng, n, base):
    out = []
    for i in range(n):
        ex = {"watch_duration": [int(rng.integers(0, 300_000))],
              "video_duration": [int(rng.integers(1, 600_000))],
              "tag": [base + i]}
        if i % 3:
            ex["extra_info"] = "xx_video_homepage_landing_yy" if i % 2 else "other"
        for s in SLOTS:
            k = int(rng.integers(0, 4))
            if k:
                ex[s] = [int(x) for x in rng.integers(0, 1 << 40, size=k)]
        out.append(ex)
    return out


def test_crc32c_known_answers():
    assert D.crc32c(b"123456789") == 0xE3069283          # the CRC-32C check value
    assert D.crc32c(b"") == 0
    assert D.crc32c(bytes(32)) == 0x8A9136AA              # RFC 3720 B.4: 32 bytes of zeros
    assert D.crc32c(bytes([0xFF] * 32)) == 0x62A8AB43     # RFC 3720 B.4: 32 bytes of 0xFF


def test_tfrecord_round_trip_and_corruption(tmp_path):
    recs = [b"", b"a", os.urandom(1000), b"xyz" * 77]
    p = str(tmp_path / "f.tfrecord")
    D.write_tfrecord(p, recs)
    assert list(D.tfrecord_iter(p)) == recs
    raw = bytearray(open(p, "rb").read())
    raw[30] ^= 0x40                                       # flip a payload bit of record 3
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ValueError, match="corrupted"):
        list(D.tfrecord_iter(p))
    assert len(list(D.tfrecord_iter(p, verify_crc=False))) == 4


def test_example_decode_matches_spec():
    rng = np.random.default_rng(1)
    exs = _examples(rng, 7, 0)
    cols = D.decode_batch([D.make_example(e) for e in exs], SLOTS)
    assert list(cols["watch_duration"]) == [e["watch_duration"][0] for e in exs]
    assert list(cols["video_duration"]) == [e["video_duration"][0] for e in exs]
    want_extra = [e.get("extra_info", "label").encode() for e in exs]   # default "label"
    assert cols["extra_info"] == want_extra
    for s in SLOTS:
        vals, splits = cols[s]
        assert splits[0] == 0 and splits.size == len(exs) + 1
        for i, e in enumerate(exs):
            assert list(vals[splits[i]:splits[i + 1]]) == e.get(s, [])
    with pytest.raises(ValueError, match="watch_duration"):
        D.decode_batch([D.make_example({"video_duration": [1]})], SLOTS)


def _write_days(root, rng, days, files_per_day, recs_per_file):
    tag = 0
    for d in days:
        os.makedirs(os.path.join(root, d), exist_ok=True)
        for k in range(files_per_day):
            exs = _examples(rng, recs_per_file, tag)
            tag += recs_per_file
            D.write_tfrecord(os.path.join(root, d, f"part-{k:03d}.tfrecord"),
                             [D.make_example(e) for e in exs])
        open(os.path.join(root, d, "_SUCCESS"), "w").close()   # not matched by the pattern
    return tag


def test_listing_sharding_interleave_batching(tmp_path):
    rng = np.random.default_rng(2)
    root = str(tmp_path)
    total = _write_days(root, rng, ["20240101", "20240102"], 5, 11)
    files = D.list_files(root, ["20240101", "missing", "20240102"], "part-*")
    assert len(files) == 10 and files == sorted(files[:5]) + sorted(files[5:])
    # every file to exactly one of 3 workers
    shards = [D.shard_files(files, 3, i) for i in range(3)]
    assert sorted(sum(shards, [])) == sorted(files)
    assert shards[1] == files[1::3]
    # interleave: cycle 4, block 8 -- the first 8 records come from file 0, the next 8 from file 1
    tag = lambda r: D.Example.FromString(r).features.feature["tag"].int64_list.value[0]  # noqa: E731
    recs = list(D.interleave(files, 4, 8, verify_crc=False))
    assert len(recs) == total
    tags = [tag(r) for r in recs]
    assert tags[:8] == list(range(0, 8)) and tags[8:16] == list(range(11, 19))
    assert sorted(tags) == list(range(total))               # nothing lost or duplicated
    bs = list(D.batch(iter(recs), 32))
    assert [len(b) for b in bs] == [32] * (total // 32) + ([total % 32] if total % 32 else [])
    reader = D.DatasetReader(shards[0], 16, SLOTS, verify_crc=True)
    n = sum(len(c["watch_duration"]) for c in reader.host_batches())
    assert n == 11 * len(shards[0])


def test_interleave_uneven_files_tf_data_order(tmp_path):
    """Files of uneven length, cycle 2, block 4: tf.data's interleave empties a slot whose file
    runs out and moves the cursor on; the next file opens only when the cursor comes back to
    that slot.  The expected order below is worked out by hand from those rules."""
    rng = np.random.default_rng(7)
    lens = [3, 10, 2, 9, 5, 4]
    names, base = [], 0
    for i, n in enumerate(lens):
        p = str(tmp_path / f"f{i}.tfrecord")
        D.write_tfrecord(p, [D.make_example(e) for e in _examples(rng, n, base)])
        names.append(p)
        base += n
    a, b, c, d, e, g = (list(range(s, s + n)) for s, n in zip(np.cumsum([0] + lens[:-1]), lens))
    want = (a[0:3] + b[0:4] + c[0:2] + b[4:8] + d[0:4] + b[8:10] + d[4:8] + e[0:4] + d[8:9]
            + e[4:5] + g[0:4])
    tag = lambda r: D.Example.FromString(r).features.feature["tag"].int64_list.value[0]  # noqa: E731
    assert [tag(r) for r in D.interleave(names, 2, 4, verify_crc=True)] == want
    assert [tag(r) for r in D.interleave(names, 1, 3, verify_crc=False)] == list(range(base))
    assert list(D.interleave([], 4, 8)) == []


@pytest.mark.gpu
def test_dataset_reader_end_to_end_labels(tmp_path):
    """dataset_reader -> parse_input_func on the GPU: labels against the CPU oracle
    (oracle/ctr_oracle.py::staytime_parse_labels, staytime/parse.py:16-71) on the decoded watch
    times and extra_info strings -- short/long, sample weight and the seconds column bit-exact,
    the soft-label bins within tests/test_labels.py's fp32-exp tolerance -- and slots as ragged
    tensors."""
    from oracle.ctr_oracle import staytime_parse_labels
    from recommendsystem_amd.parse import MODEL_PREFIX
    bins = [-19.0 + 0.5 * i for i in range(400)]     # staytime/config.py:18 bin_list
    rng = np.random.default_rng(3)
    root = str(tmp_path)
    _write_days(root, rng, ["d1"], 3, 20)
    reader = D.dataset_reader(root, ["d1"], "part-*", 25, slots=SLOTS, shard_num=1, shard_id=0)
    host = list(reader.host_batches())
    got = list(reader)
    assert len(got) == len(host) == 3
    for cols, (feat, y, sw) in zip(host, got):
        info = [e.decode() for e in cols["extra_info"]]
        stay, short, long_, sw_ref = staytime_parse_labels(cols["watch_duration"], info, bins)
        assert np.any(sw_ref == 5) and np.any(sw_ref == 1)
        got = y[f"{MODEL_PREFIX}_staytime"].cpu().numpy().reshape(stay.shape)
        np.testing.assert_array_equal(got[:, -1], stay[:, -1])
        err = np.abs(got[:, :400] - stay[:, :400])
        assert (err <= 1e-8 + 4e-7 * np.abs(stay[:, :400])).all(), err.max()
        np.testing.assert_array_equal(y[f"{MODEL_PREFIX}_shortplay"].cpu().numpy().reshape(-1), short)
        np.testing.assert_array_equal(y[f"{MODEL_PREFIX}_longplay"].cpu().numpy().reshape(-1), long_)
        np.testing.assert_array_equal(sw.cpu().numpy().reshape(-1), sw_ref)
        for s in SLOTS:
            v, sp = feat[s]
            assert v.is_cuda and torch.equal(v.cpu(), torch.from_numpy(cols[s][0]))
            assert torch.equal(sp.cpu(), torch.from_numpy(cols[s][1]))
        assert feat["example_id"] == cols["extra_info"]
