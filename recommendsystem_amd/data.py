"""staytime ``dataset_reader`` (``staytime/parse.py:73-92``): TFRecord files of
``tf.train.Example`` -> per-worker file shard -> interleave -> batch -> ``parse_input_func``
(labels on the GPU) -> prefetch, without TensorFlow.

    dataset_reader(data_dir, dates, match_pattern, batch_size)        # parse.py:73
        files   = list_files(data_dir, days=dates, match_pattern)     # tn.data.list_files
        files   = files[shard_id::shard_num]                          # .shard(shard_num, id)
        records = interleave(files, cycle_length=4, block_length=8)   # .interleave(TFRecordDataset)
        batches = batch(records, batch_size)                          # .batch
        -> parse_input_func(decode(batch))                            # .map(parse_input_func)
        -> background prefetch into pinned host memory + async H2D    # .prefetch(AUTOTUNE)

Pinned decisions (tensornet / tf.data internals are not in the reference):
  * ``list_files``: ``data_dir/<day>/`` for each day in ``days`` (in the given order), the file
    names matching the glob ``match_pattern``, sorted; a day without a directory contributes
    nothing.  (tn.data.list_files is not vendored; this is the layout its call site implies.)
  * shard: file i goes to worker ``i % shard_num`` (tf.data ``shard`` on the file list); the
    defaults ``shard_num / shard_id`` are torch.distributed's world size / rank (tn.core).
  * interleave: tf.data's deterministic order -- ``cycle_length`` files open, ``block_length``
    consecutive records from each in turn; an exhausted file's slot takes the next file.
  * batch: consecutive ``batch_size`` records, the last partial batch kept (drop_remainder=False).
  * TFRecord framing: uint64 length, uint32 masked CRC32C of the length, payload, uint32 masked
    CRC32C of the payload (both checked unless ``verify_crc=False``).
  * Example decoding (``tf.io.parse_example`` with the reference's feature spec, parse.py:17-23):
    ``extra_info`` bytes, default "label"; ``video_duration`` / ``watch_duration`` int64
    (required); every slot a VarLen int64 list -> ``(values, row_splits)``.
The host does framing, protobuf decoding and the extra_info regex; the label math runs on the GPU
(``parse.parse_input_func``).
"""
from __future__ import annotations

import fnmatch
import os
import queue
import struct
import threading
from typing import Iterable, Iterator, Sequence

import numpy as np
import torch

from .parse import MODEL_PREFIX, parse_input_func

# ---------------------------------------------------------------------------------------------
# CRC32C (Castagnoli, reflected polynomial 0x82F63B78) and TFRecord's mask
# ---------------------------------------------------------------------------------------------
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)
del _i, _c


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    t = _CRC_TABLE
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def tfrecord_iter(path: str, verify_crc: bool = True) -> Iterator[bytes]:
    """The records of one TFRecord file."""
    with open(path, "rb") as f:
        while True:
            head = f.read(12)
            if not head:
                return
            if len(head) != 12:
                raise ValueError(f"{path}: truncated record header")
            n, lcrc = struct.unpack("<QI", head)
            if verify_crc and masked_crc32c(head[:8]) != lcrc:
                raise ValueError(f"{path}: corrupted record length")
            data = f.read(n)
            tail = f.read(4)
            if len(data) != n or len(tail) != 4:
                raise ValueError(f"{path}: truncated record")
            if verify_crc and masked_crc32c(data) != struct.unpack("<I", tail)[0]:
                raise ValueError(f"{path}: corrupted record payload")
            yield data


def write_tfrecord(path: str, records: Iterable[bytes]) -> None:
    """TFRecord writer (fixtures and tools)."""
    with open(path, "wb") as f:
        for r in records:
            ln = struct.pack("<Q", len(r))
            f.write(ln + struct.pack("<I", masked_crc32c(ln)) + r +
                    struct.pack("<I", masked_crc32c(r)))


# ---------------------------------------------------------------------------------------------
# tf.train.Example (tensorflow/core/example/{example,feature}.proto), built at import time
# ---------------------------------------------------------------------------------------------
def _example_classes():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fd = descriptor_pb2.FileDescriptorProto(name="rs_tf_example.proto", package="rs_tf",
                                            syntax="proto3")
    L = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields, oneofs=()):
        m = fd.message_type.add(name=name)
        for o in oneofs:
            m.oneof_decl.add(name=o)
        for fname, num, ftype, label, tname, oneof in fields:
            fld = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                fld.type_name = tname
            if oneof is not None:
                fld.oneof_index = oneof
        return m

    rep, opt = L.LABEL_REPEATED, L.LABEL_OPTIONAL
    msg("BytesList", [("value", 1, L.TYPE_BYTES, rep, None, None)])
    msg("FloatList", [("value", 1, L.TYPE_FLOAT, rep, None, None)])
    msg("Int64List", [("value", 1, L.TYPE_INT64, rep, None, None)])
    msg("Feature", [("bytes_list", 1, L.TYPE_MESSAGE, opt, ".rs_tf.BytesList", 0),
                    ("float_list", 2, L.TYPE_MESSAGE, opt, ".rs_tf.FloatList", 0),
                    ("int64_list", 3, L.TYPE_MESSAGE, opt, ".rs_tf.Int64List", 0)], oneofs=("kind",))
    feats = msg("Features", [("feature", 1, L.TYPE_MESSAGE, rep, ".rs_tf.Features.FeatureEntry", None)])
    entry = feats.nested_type.add(name="FeatureEntry")
    entry.field.add(name="key", number=1, type=L.TYPE_STRING, label=opt)
    entry.field.add(name="value", number=2, type=L.TYPE_MESSAGE, label=opt, type_name=".rs_tf.Feature")
    entry.options.map_entry = True
    msg("Example", [("features", 1, L.TYPE_MESSAGE, opt, ".rs_tf.Features", None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = getattr(message_factory, "GetMessageClass", None)
    if get is None:  # older protobuf
        factory = message_factory.MessageFactory(pool)
        get = lambda d: factory.GetPrototype(d)  # noqa: E731
    return get(pool.FindMessageTypeByName("rs_tf.Example")), get(pool.FindMessageTypeByName("rs_tf.Feature"))


Example, Feature = _example_classes()


def make_example(features: dict) -> bytes:
    """Serialize {name: bytes | str | [int] | [float]} as a tf.train.Example (fixtures)."""
    ex = Example()
    for k, v in features.items():
        f = ex.features.feature[k]
        if isinstance(v, (bytes, str)):
            f.bytes_list.value.append(v.encode() if isinstance(v, str) else v)
        elif isinstance(v, (list, tuple, np.ndarray)) and len(v) and isinstance(np.asarray(v).flat[0], (float, np.floating)):
            f.float_list.value.extend(float(x) for x in v)
        else:
            f.int64_list.value.extend(int(x) for x in np.atleast_1d(v))
    return ex.SerializeToString()


def decode_batch(records: Sequence[bytes], slots: Sequence[str]) -> dict:
    """tf.io.parse_example with parse.py:17-23's spec -> the decoded columns parse_input_func
    takes (VarLen slots as (values int64, row_splits int64))."""
    B = len(records)
    extra, vdur, wdur = [], np.empty(B, np.int64), np.empty(B, np.int64)
    vals = {s: [] for s in slots}
    lens = {s: np.zeros(B, np.int64) for s in slots}
    for i, r in enumerate(records):
        ex = Example()
        ex.ParseFromString(r)
        fm = ex.features.feature
        extra.append(fm["extra_info"].bytes_list.value[0] if "extra_info" in fm and
                     len(fm["extra_info"].bytes_list.value) else b"label")
        for name, arr in (("video_duration", vdur), ("watch_duration", wdur)):
            if name not in fm or len(fm[name].int64_list.value) != 1:
                raise ValueError(f"record {i}: FixedLenFeature {name} (int64, no default) missing")
            arr[i] = fm[name].int64_list.value[0]
        for s in slots:
            if s in fm:
                v = fm[s].int64_list.value
                vals[s].extend(v)
                lens[s][i] = len(v)
    out = {"extra_info": extra, "video_duration": vdur, "watch_duration": wdur}
    for s in slots:
        out[s] = (np.asarray(vals[s], dtype=np.int64),
                  np.concatenate([[0], np.cumsum(lens[s])]).astype(np.int64))
    return out


# ---------------------------------------------------------------------------------------------
# file listing, sharding, interleave, batching
# ---------------------------------------------------------------------------------------------
def list_files(data_dir: str, days: Sequence[str], match_pattern: str = "*") -> list[str]:
    out = []
    for d in days:
        dd = os.path.join(data_dir, str(d))
        if os.path.isdir(dd):
            out += [os.path.join(dd, n) for n in sorted(os.listdir(dd))
                    if fnmatch.fnmatch(n, match_pattern) and os.path.isfile(os.path.join(dd, n))]
    return out


def shard_files(files: Sequence[str], shard_num: int, shard_id: int) -> list[str]:
    if not 0 <= shard_id < shard_num:
        raise ValueError(f"shard_id {shard_id} outside [0, {shard_num})")
    return list(files[shard_id::shard_num])


def interleave(files: Sequence[str], cycle_length: int = 4, block_length: int = 8,
               verify_crc: bool = True) -> Iterator[bytes]:
    """``Dataset.from_tensor_slices(files).interleave(TFRecordDataset, cycle_length,
    block_length)`` in its deterministic order (staytime/parse.py:80-84; the parallel form with
    ``deterministic`` order yields the sequential order).  tf.data's interleave keeps
    ``cycle_length`` slots and a cursor: an open slot yields up to ``block_length`` records and
    the cursor moves on; a slot whose file runs out is emptied and the cursor moves on at once; an
    empty slot the cursor reaches takes the next pending file (while any remain) and reads from
    it, otherwise it is skipped."""
    if cycle_length < 1 or block_length < 1:
        raise ValueError("cycle_length and block_length must be >= 1")
    pending = list(files)
    slots: list = [None] * cycle_length
    n_open, k, blk = 0, 0, 0
    while pending or n_open:
        it = slots[k]
        if it is None:
            if pending:
                slots[k] = tfrecord_iter(pending.pop(0), verify_crc)
                n_open += 1
            else:
                k, blk = (k + 1) % cycle_length, 0
            continue
        try:
            rec = next(it)
        except StopIteration:
            slots[k] = None
            n_open -= 1
            k, blk = (k + 1) % cycle_length, 0
            continue
        yield rec
        blk += 1
        if blk == block_length:
            k, blk = (k + 1) % cycle_length, 0


def batch(records: Iterator[bytes], batch_size: int) -> Iterator[list[bytes]]:
    cur: list[bytes] = []
    for r in records:
        cur.append(r)
        if len(cur) == batch_size:
            yield cur
            cur = []
    if cur:
        yield cur


def _pin(cols: dict) -> dict:
    """numpy columns -> pinned host tensors (async H2D in parse_input_func)."""
    out = {}
    for k, v in cols.items():
        if k == "extra_info":
            out[k] = v
        elif isinstance(v, tuple):
            out[k] = tuple(torch.from_numpy(np.ascontiguousarray(a)).pin_memory() for a in v)
        else:
            out[k] = torch.from_numpy(np.ascontiguousarray(v)).pin_memory()
    return out


class DatasetReader:
    """Iterable of parse_input_func triples; decoding and pinning run on a background thread
    ``prefetch`` batches ahead; the H2D copies and the label kernel are issued by the consumer
    (on its current stream) when it takes the batch."""

    def __init__(self, files: Sequence[str], batch_size: int, slots: Sequence[str],
                 cycle_length: int = 4, block_length: int = 8, prefetch: int = 2,
                 device: str | torch.device = "cuda", prefix: str = MODEL_PREFIX,
                 verify_crc: bool = True):
        self.files, self.batch_size, self.slots = list(files), int(batch_size), list(slots)
        self.cycle_length, self.block_length = cycle_length, block_length
        self.prefetch, self.device, self.prefix, self.verify_crc = prefetch, device, prefix, verify_crc

    def host_batches(self) -> Iterator[dict]:
        """Decoded (unpinned numpy) batches in order: the loader without the device half."""
        recs = interleave(self.files, self.cycle_length, self.block_length, self.verify_crc)
        for b in batch(recs, self.batch_size):
            yield decode_batch(b, self.slots)

    def __iter__(self):
        q: queue.Queue = queue.Queue(maxsize=max(1, self.prefetch))
        stop = threading.Event()
        err: list = []

        def work():
            try:
                for cols in self.host_batches():
                    if stop.is_set():
                        return
                    q.put(_pin(cols) if torch.cuda.is_available() else cols)
            except BaseException as e:  # surfaced in the consumer
                err.append(e)
            finally:
                q.put(None)

        th = threading.Thread(target=work, daemon=True)
        th.start()
        try:
            while True:
                cols = q.get()
                if cols is None:
                    break
                yield parse_input_func(cols, device=self.device, prefix=self.prefix)
        finally:
            stop.set()
            while th.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    pass
                th.join(timeout=0.05)
        if err:
            raise err[0]


def dataset_reader(data_dir: str, dates: Sequence[str], match_pattern: str, batch_size: int,
                   slots: Sequence[str] | None = None, shard_num: int | None = None,
                   shard_id: int | None = None, **kw) -> DatasetReader:
    """staytime/parse.py:73-92.  ``slots`` defaults to the staytime Config.SLOTS set
    (feature_config.STAYTIME_SLOTS); shard_num / shard_id default to the torch.distributed world size /
    rank (tn.core.shard_num() / self_shard_id())."""
    if shard_num is None or shard_id is None:
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            shard_num, shard_id = torch.distributed.get_world_size(), torch.distributed.get_rank()
        else:
            shard_num, shard_id = 1, 0
    if slots is None:
        from .feature_config import STAYTIME_SLOTS
        slots = sorted(set(STAYTIME_SLOTS))          # parse.py:22: for slot in set(C.SLOTS)
    files = shard_files(list_files(data_dir, dates, match_pattern), shard_num, shard_id)
    return DatasetReader(files, batch_size, slots, **kw)
