"""Examples as bytes (sk_dataset_export / sk_dataset_import) and the host
pack digest (sk_dataset_pack_digest): a dataset rebuilt from the bytes of
another -- whole, or from shares appended in order -- packs to the same
arrays bit for bit, which is what lets ranks build shares of a dataset and
gather them (shard.build_split; the world-2 test is in test_distributed.py).
CPU only: building, exporting and packing run on the host."""
import ctypes as C

import numpy as np
import pytest

import stem_kernel_amd as ska
from stem_kernel_amd._lib import lib


@pytest.fixture(scope="module")
def seqs():
    return ska.random_sequences(9, 90, 0x5EED0011) + ska.random_sequences(3, 37, 5)


def test_round_trip_packs_identically(seqs):
    a = ska.Dataset.synthetic(seqs, labels=["+1" if k % 3 else "-1" for k in range(len(seqs))])
    b = ska.Dataset().import_bytes(a.export())
    assert len(b) == len(a)
    for i in range(len(a)):
        assert b.label(i) == a.label(i)
        da, db = a.dag(i), b.dag(i)
        for k in da:
            assert np.array_equal(da[k], db[k]), (i, k)
        pa, na = a.profile(i)
        pb, nb = b.profile(i)
        assert np.array_equal(pa, pb) and na == nb
        for u, v in zip(a.bpla_weights(i), b.bpla_weights(i)):
            assert np.array_equal(u, v)
    assert a.pack_digest() == b.pack_digest()


def test_shares_in_order_pack_as_the_whole(seqs):
    whole = ska.Dataset.synthetic(seqs)
    n = len(seqs)
    cuts = [0, 4, 5, 11, n]
    out = ska.Dataset()
    for lo, hi in zip(cuts, cuts[1:]):
        out.import_bytes(ska.Dataset.synthetic(seqs[lo:hi]).export())
    assert out.pack_digest() == whole.pack_digest()
    # a different order is a different dataset
    rev = ska.Dataset()
    for lo, hi in reversed(list(zip(cuts, cuts[1:]))):
        rev.import_bytes(ska.Dataset.synthetic(seqs[lo:hi]).export())
    assert rev.pack_digest() != whole.pack_digest()


def test_alignments_round_trip():
    base = ska.random_sequences(3, 60, 0x5EED0012)
    alns = [[s, s[:30] + "-" * 5 + s[35:], s[::-1]] for s in base]
    a = ska.Dataset.synthetic_alignments(alns)
    b = ska.Dataset().import_bytes(a.export(1, 2))
    assert len(b) == 2
    for i in range(2):
        assert np.array_equal(a.profile(i + 1)[0], b.profile(i)[0])
        assert a.shape(i + 1) == b.shape(i)


def test_malformed_buffers_append_nothing(seqs):
    a = ska.Dataset.synthetic(seqs[:3])
    data = a.export()
    b = ska.Dataset.synthetic(seqs[3:4])
    for bad in (data[:-1], data[:40], b"XXXX" + data[4:], data + b"\0"):
        with pytest.raises(RuntimeError):
            b.import_bytes(bad)
        assert len(b) == 1
    b.import_bytes(ska.Dataset().export())  # zero examples
    assert len(b) == 1


def test_inconsistent_examples_rejected(seqs):
    """A well-framed buffer whose example breaks the builder's invariants
    (here: its length no longer matches its rows and profile) appends
    nothing."""
    a = ska.Dataset.synthetic(seqs[:2], labels=["+1", "-1"])
    data = bytearray(a.export())
    lab = int.from_bytes(data[12:16], "little")
    off = 16 + lab  # example 0's len (int32) after the header and its label
    L = int.from_bytes(data[off:off + 4], "little", signed=True)
    assert L == len(seqs[0])
    data[off:off + 4] = (L + 1).to_bytes(4, "little", signed=True)
    b = ska.Dataset()
    with pytest.raises(RuntimeError):
        b.import_bytes(data)
    assert len(b) == 0
    # no bp information (MData(ma)): no DAG, still a valid example
    ds = ska.Dataset()
    ds.add("+1", [seqs[0]], None, use_bp=False)
    assert len(ska.Dataset().import_bytes(ds.export())) == 1


def test_export_bounds_and_short_buffer(seqs):
    a = ska.Dataset.synthetic(seqs[:2])
    need = C.c_size_t()
    assert lib().sk_dataset_export(a._h, 1, 2, None, 0, C.byref(need)) != 0  # past the end
    assert lib().sk_dataset_export(a._h, 0, 2, None, 0, C.byref(need)) == 0
    buf = C.create_string_buffer(need.value)
    assert lib().sk_dataset_export(a._h, 0, 2, buf, need.value - 1, C.byref(need)) != 0  # SK_ERR_RANGE
