"""TFRecord/Example codec and the lib/dataset.py drop-in (host logic, CPU)."""
import os

import numpy as np
import pytest


def test_example_roundtrip_and_record_container(tmp_path):
    from jr import tfrecord
    ex = {"image/encoded": b"\xff\xd8jpeg-bytes", "image/format": b"jpeg", "image/class/label": 1,
          "image/height": 299, "image/width": 299, "neg": [-5, 2 ** 40], "f": [0.5, 1.25]}
    data = tfrecord.encode_example(ex)
    back = tfrecord.decode_example(data)
    assert back["image/encoded"] == [ex["image/encoded"]]
    assert back["image/class/label"] == [1] and back["image/height"] == [299]
    assert back["neg"] == [-5, 2 ** 40] and back["f"] == [0.5, 1.25]
    path = str(tmp_path / "a.tfrecord")
    with tfrecord.TFRecordWriter(path) as w:
        w.write(data)
        w.write(b"")
        w.write(b"x" * 100000)
    recs = list(tfrecord.read_records(path))
    assert recs == [data, b"", b"x" * 100000]
    raw = bytearray(open(path, "rb").read())
    raw[20] ^= 1                                   # corrupt the first payload
    open(path, "wb").write(bytes(raw))
    with pytest.raises(tfrecord.TFRecordError):
        list(tfrecord.read_records(path))


@pytest.fixture(scope="module")
def records(tmp_path_factory):
    from jr import synth_records
    d = str(tmp_path_factory.mktemp("tfr"))
    synth_records.write_split(d, 21, size=64, num_shards=3, name="train")
    open(os.path.join(d, "notes.txt"), "w").write("ignored: wrong extension")
    return d


def test_dataset_shapes_order_and_partial_batch(records):
    import lib.dataset as D
    from jr import synth
    ds = D.initialize_dataset(records, 8, image_dim=[64, 64])
    batches = list(ds)
    assert [len(b[0]) for b in batches] == [8, 8, 5]              # partial last batch kept
    x, y = batches[0]
    assert x.dtype == np.float32 and x.shape == (8, 64, 64, 3) and y.shape == (8, 1)
    assert x.max() <= 1.0 and x.min() >= 0.0
    # os.listdir order of the shard files (lib/dataset.py:5-8)
    files = [n for n in os.listdir(records) if n.endswith(".tfrecord")]
    assert [os.path.basename(f) for f in ds.files] == files
    # label values come from the records; JPEG q=100 keeps pixels close
    allx = np.concatenate([b[0] for b in batches])
    ally = np.concatenate([b[1] for b in batches])
    idx = []
    for f in files:                                 # shard s holds images [7s, 7s+7)
        s = int(f.split("-")[1])
        idx += list(range(7 * s, 7 * s + 7))
    want_y = synth.labels(0, 21)[idx]
    np.testing.assert_array_equal(ally, want_y)
    # JPEG q=100 (4:2:0 chroma) keeps the decoded pixels close to the source
    # image they came from, and far from any other image of the set
    errs = [np.mean(np.abs(allx[0] - synth.fundus_image(k, 64).astype(np.float32) / 255)) for k in range(21)]
    assert int(np.argmin(errs)) == idx[0] and errs[idx[0]] < 8.0 / 255


def test_uint8_mode_is_bitwise_scaled_float(records):
    import lib.dataset as D
    a = np.concatenate([b[0] for b in D.initialize_dataset(records, 4, image_dim=[64, 64])])
    u = np.concatenate([b[0] for b in D.initialize_dataset(records, 4, image_dim=[64, 64], decode_dtype="uint8")])
    assert u.dtype == np.uint8
    np.testing.assert_array_equal(u.astype(np.float32) * np.float32(1 / 255), a)


def test_shuffle_is_a_permutation_and_seedable(records):
    import lib.dataset as D
    base = np.concatenate([b[1] for b in D.initialize_dataset(records, 4, image_dim=[64, 64])])
    s1 = D.initialize_dataset(records, 4, image_dim=[64, 64], shuffle_buffer_size=8, seed=5, num_workers=3,
                              prefetch_buffer_size=8)
    a = [b[0].sum(axis=(1, 2, 3)) for b in s1]
    b_ = [b[0].sum(axis=(1, 2, 3)) for b in D.initialize_dataset(records, 4, image_dim=[64, 64],
                                                                  shuffle_buffer_size=8, seed=5)]
    np.testing.assert_array_equal(np.concatenate(a), np.concatenate(b_))
    assert sorted(np.concatenate([b[1] for b in s1]).ravel().tolist()) == sorted(base.ravel().tolist())
    plain = np.concatenate([b[0].sum(axis=(1, 2, 3)) for b in D.initialize_dataset(records, 4, image_dim=[64, 64])])
    assert not np.array_equal(np.concatenate(a), plain)
    # re-iterating reshuffles (reshuffle_each_iteration) but keeps the multiset
    again = np.concatenate([b[0].sum(axis=(1, 2, 3)) for b in s1])
    np.testing.assert_allclose(np.sort(again), np.sort(plain))


def test_repeat_epochs_and_channels_first_is_a_reshape(records):
    import lib.dataset as D
    ds = D.initialize_dataset(records, 10, num_epochs=2, image_dim=[64, 64])
    assert [len(b[0]) for b in ds] == [10, 10, 10, 10, 2]
    cl = next(iter(D.initialize_dataset(records, 2, image_dim=[64, 64])))[0]
    cf = next(iter(D.initialize_dataset(records, 2, image_dim=[64, 64], image_data_format="channels_first")))[0]
    assert cf.shape == (2, 3, 64, 64)
    np.testing.assert_array_equal(cf.reshape(cl.shape), cl)       # App. C Q3: reshape, not transpose
    with pytest.raises(TypeError):
        D.initialize_dataset(records, 2, image_data_format="nchw")
