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


# ---- native record index / Example parse (jr_tfrecord_index, jr_example_parse_image)
# checked against the pure-Python restatement of the same wire formats
# (jr.tfrecord.read_records / decode_example) and the per-record element
# function lib.dataset._parse_example.

def _vint(v):
    from jr import tfrecord
    return tfrecord._varint(v)


def _ex(entries):
    """Example bytes from raw (name, Feature payload) map entries, in order."""
    from jr import tfrecord as T
    body = b"".join(T._field(1, 2, T._field(1, 2, n.encode()) + T._field(2, 2, f)) for n, f in entries)
    return T._field(1, 2, body)


def _bytes_feat(*vals):
    from jr import tfrecord as T
    return T._field(1, 2, b"".join(T._field(1, 2, v) for v in vals))


def _int_feat(*vals, packed=True):
    from jr import tfrecord as T
    if packed:
        return T._field(3, 2, T._field(1, 2, b"".join(_vint(v & (2 ** 64 - 1)) for v in vals)))
    return T._field(3, 2, b"".join(bytes([1 << 3]) + _vint(v & (2 ** 64 - 1)) for v in vals))


def _good(label=1, packed=True):
    return [("image/encoded", _bytes_feat(b"\xff\xd8JPEGDATA")), ("image/format", _bytes_feat(b"jpeg")),
            ("image/class/label", _int_feat(label, packed=packed)), ("image/height", _int_feat(299)),
            ("image/width", _int_feat(299))]


def test_native_index_matches_python_reader_and_stops_at_damage(tmp_path):
    from jr import tfrecord
    recs = [b"", b"a", b"x" * 100003] + [bytes([i]) * (i * 37) for i in range(40)]
    path = str(tmp_path / "r.tfrecord")
    with tfrecord.TFRecordWriter(path) as w:
        for r in recs:
            w.write(r)
    f = tfrecord.RecordFile(path, parse=False)
    assert f.error is None and f.num_records == len(recs)
    assert [f.record(i) for i in range(f.num_records)] == list(tfrecord.read_records(path)) == recs
    raw = bytearray(open(path, "rb").read())
    bad_at = 12 + 0 + 4 + 12 + 1 + 4 + 12 + 50      # inside the third payload
    raw[bad_at] ^= 0x40
    open(path, "wb").write(bytes(raw))
    f = tfrecord.RecordFile(path, parse=False)
    assert f.num_records == 2 and "corrupted record data" in f.error
    with pytest.raises(tfrecord.TFRecordError):
        f.raise_if_damaged()
    assert tfrecord.RecordFile(path, verify=False, parse=False).num_records == len(recs)
    open(path, "wb").write(bytes(raw[:-3]))           # truncated tail
    f = tfrecord.RecordFile(path, verify=False, parse=False)
    assert f.num_records == len(recs) - 1 and "truncated" in f.error
    empty = str(tmp_path / "e.tfrecord")
    open(empty, "wb").close()
    assert tfrecord.RecordFile(empty).num_records == 0


def test_native_example_parse_matches_python_decoder(tmp_path):
    from jr import tfrecord
    cases = [
        (_ex(_good(1)), 0),
        (_ex(_good(0, packed=False)), 0),
        (_ex(_good(-7)), 0),                                          # negative int64 label
        (_ex(_good(1)[:2] + _good(1)[3:]), 4),                        # label missing
        (_ex(_good(1)[:1] + [("image/format", _bytes_feat())] + _good(1)[2:]), 2),   # zero values
        (_ex(_good(1)[:2] + [("image/class/label", _int_feat(0, 1))] + _good(1)[3:]), 4),  # two values
        (_ex(_good(1)[:3] + [("image/height", _bytes_feat(b"299"))] + _good(1)[4:]), 8),  # wrong kind
        (_ex(_good(1) + [("image/class/label", _int_feat(5))]), 0),  # duplicate key: last wins
        (_ex([("extra", _int_feat(3, 4, 5))] + _good(1)), 0),        # unrelated features skipped
        (b"\x0a\xff\xff", -1),                                        # truncated protobuf
        (b"", 31),                                                    # empty Example: all missing
    ]
    path = str(tmp_path / "p.tfrecord")
    with tfrecord.TFRecordWriter(path) as w:
        for data, _ in cases:
            w.write(data)
    f = tfrecord.RecordFile(path)
    assert list(f.status) == [st for _, st in cases]
    for i, (data, st) in enumerate(cases):
        if st == -1:
            continue
        ex = tfrecord.decode_example(data)
        if st & 1 == 0:
            assert bytes(f.encoded(i)) == ex["image/encoded"][0]
        if st & 4 == 0:
            assert int(f.label[i]) == ex["image/class/label"][0]
        if st == 0:
            assert int(f.height[i]) == ex["image/height"][0] == 299 and int(f.width[i]) == 299
    with pytest.raises(ValueError, match="image/class/label"):
        f.check(3)
    with pytest.raises(ValueError, match="not a serialized"):
        f.check(9)
    assert int(f.label[7]) == 5


def test_dataset_matches_per_record_python_path(records):
    """Native-index pipeline (any worker count) == the per-record element
    function over tfrecord.read_records, bit for bit, both decode dtypes."""
    import lib.dataset as D
    from jr import tfrecord
    for dtype in ("float32", "uint8"):
        want_x, want_y = [], []
        for path in D._tfrecord_files_from_folder(records):
            for rec in tfrecord.read_records(path):
                x, y = D._parse_example(rec, [64, 64, 3], dtype)
                want_x.append(x)
                want_y.append(y)
        for nw in (1, 3):
            got = list(D.initialize_dataset(records, 5, image_dim=[64, 64], num_workers=nw, decode_dtype=dtype,
                                            prefetch_buffer_size=10))
            np.testing.assert_array_equal(np.concatenate([g[0] for g in got]), np.stack(want_x))
            np.testing.assert_array_equal(np.concatenate([g[1] for g in got]), np.stack(want_y))


def test_damaged_file_delivers_records_before_the_damage(tmp_path):
    import lib.dataset as D
    from jr import synth_records, tfrecord
    d = str(tmp_path)
    synth_records.write_split(d, 9, size=32, num_shards=1, name="train")
    path = os.path.join(d, os.listdir(d)[0])
    f = tfrecord.RecordFile(path)
    raw = bytearray(open(path, "rb").read())
    raw[int(f.offsets[6]) + 10] ^= 1                  # corrupt record 6
    del f
    open(path, "wb").write(bytes(raw))
    got = []
    with pytest.raises(tfrecord.TFRecordError):
        for x, _ in D.initialize_dataset(d, 2, image_dim=[32, 32]):
            got.append(len(x))
    assert got == [2, 2, 2]                           # records 0-5, then DataLoss at record 6


def test_shards_partition_the_stream_and_decode_only_their_batches(records, monkeypatch):
    """shard=(rank, world): the ranks' batches are exactly the single-process
    batches b % world == rank, in order, over several seeded-shuffle epochs,
    and each rank decodes only its own batches (JPEG work split, not
    repeated)."""
    import lib.dataset as D
    calls = []
    real = D.Dataset._decode
    monkeypatch.setattr(D.Dataset, "_decode", lambda self, data, dst: (calls.append(1), real(self, data, dst))[1])
    kw = dict(image_dim=[64, 64], shuffle_buffer_size=16, seed=9, decode_dtype="uint8")
    full = D.initialize_dataset(records, 4, **kw)
    ref = [list(full) for _ in range(2)]                       # two epochs
    world = 3
    for rank in range(world):
        ds = D.initialize_dataset(records, 4, shard=(rank, world), **kw)
        for epoch in range(2):
            calls.clear()
            got = list(ds)
            want = ref[epoch][rank::world]
            assert len(got) == len(want)
            for (x, y), (wx, wy) in zip(got, want):
                np.testing.assert_array_equal(x, wx)
                np.testing.assert_array_equal(y, wy)
            assert len(calls) == sum(len(b[0]) for b in want)  # own batches only
    with pytest.raises(ValueError):
        D.initialize_dataset(records, 4, shard=(2, 2))


def test_seeded_epochs_agree_after_an_early_stop(records):
    """A rank that stops an epoch early (capped steps) still shuffles the
    next epoch like the others: epoch k's order depends on (seed, k) only."""
    import lib.dataset as D
    kw = dict(image_dim=[64, 64], shuffle_buffer_size=16, seed=4, decode_dtype="uint8")
    a, b = D.initialize_dataset(records, 4, **kw), D.initialize_dataset(records, 4, **kw)
    it = iter(a)
    next(it)                                                  # epoch 0 cut short
    D.close_iterator(it)
    list(b)                                                   # epoch 0 in full
    for (x, _), (y, _) in zip(a, b):                          # epoch 1
        np.testing.assert_array_equal(x, y)


def test_prefetch_close_stops_the_pipeline(records):
    """close() after an early break ends the prefetch thread and shuts the
    decode pool down (no per-epoch thread leak)."""
    import threading
    import lib.dataset as D
    ds = D.initialize_dataset(records, 2, image_dim=[64, 64], prefetch_buffer_size=4)
    before = threading.active_count()
    for _ in range(3):
        it = iter(ds)
        next(it)
        D.close_iterator(it)
        it.join(timeout=10)
        assert not it._t.is_alive()
        with pytest.raises(StopIteration):
            next(it)
    assert threading.active_count() <= before + 1


def test_native_jpeg_decoder(records):
    """libjr_jpeg (IJG libjpeg 9 entropy decode + IDCT, then libjpeg-turbo's
    fancy upsampling and fixed-point colour conversion restated in
    jr_jpeg.cpp; outside the GIL).  With the same IDCT (ISLOW) the pixels are
    BIT-IDENTICAL to Pillow's libjpeg-turbo decode for 4:4:4, 4:2:2 and 4:2:0
    files, odd sizes included (edge columns / rows of the triangle filter).
    (Linking libjpeg 9's own output path instead differs by up to 65 LSB on
    4:2:0: it scales the chroma IDCT up rather than upsampling.)  TF's default
    IFAST IDCT stays within a few LSB of ISLOW.  The pipeline decodes in place
    either way and its labels / shapes are unchanged."""
    import io
    from PIL import Image
    import lib.dataset as D
    from jr import jpeg as J
    if not J.available():
        pytest.skip("libjr_jpeg.so not built")
    rng = np.random.default_rng(0)
    fast_dev = []
    for h, w in ((61, 77), (64, 64), (17, 33), (1, 9)):
        img = np.clip(rng.normal(120, 40, (h, w, 3)), 0, 255).astype(np.uint8)
        for sub in (0, 1, 2):                                 # 4:4:4, 4:2:2, 4:2:0
            buf = io.BytesIO()
            Image.fromarray(img).save(buf, "JPEG", quality=95, subsampling=sub)
            data = buf.getvalue()
            pil = D.decode_jpeg(data).astype(int)
            islow = J.decode(data, "islow").astype(int)
            ifast = J.decode(data, "ifast").astype(int)
            assert islow.shape == pil.shape == (h, w, 3)
            assert np.array_equal(islow, pil), (h, w, sub, np.abs(islow - pil).max())
            assert np.abs(ifast - islow).max() <= 8
            fast_dev.append(np.abs(ifast - islow).ravel())
    assert np.concatenate(fast_dev).mean() < 1.0
    # 4:4:0 (h1v2 chroma, e.g. a losslessly transposed 4:2:2 file): Pillow
    # cannot write it, IJG's cjpeg (same image, /opt/conda) can; libjpeg-turbo's
    # vertical-only triangle filter (the h2v2 path was taken and
    # stretched the left half of the chroma row)
    import shutil
    import subprocess
    cjpeg = shutil.which("cjpeg") or ("/opt/conda/bin/cjpeg" if os.path.exists("/opt/conda/bin/cjpeg") else None)
    if cjpeg:
        for h, w in ((61, 77), (64, 64), (1, 9), (2, 5)):
            img = np.clip(rng.normal(120, 40, (h, w, 3)), 0, 255).astype(np.uint8)
            ppm = b"P6\n%d %d\n255\n" % (w, h) + img.tobytes()
            data = subprocess.run([cjpeg, "-quality", "95", "-sample", "1x2,1x1,1x1"], input=ppm,
                                  capture_output=True, check=True).stdout
            im = Image.open(io.BytesIO(data))
            assert [s[1:3] for s in im.layer] == [(1, 2), (1, 1), (1, 1)]
            pil = np.asarray(im.convert("RGB")).astype(int)
            islow = J.decode(data, "islow").astype(int)
            assert np.array_equal(islow, pil), (h, w, np.abs(islow - pil).max())
    gray = io.BytesIO()
    g = np.clip(rng.normal(120, 40, (61, 77)), 0, 255).astype(np.uint8)
    Image.fromarray(g).save(gray, "JPEG", quality=90)
    dg = J.decode(gray.getvalue(), "islow")
    assert dg.shape == (61, 77, 1)
    np.testing.assert_array_equal(dg[..., 0], np.asarray(Image.open(io.BytesIO(gray.getvalue()))))
    with pytest.raises(ValueError):
        J.decode(b"\xff\xd8 not a jpeg")
    kw = dict(image_dim=[64, 64], decode_dtype="uint8")
    a = list(D.initialize_dataset(records, 8, jpeg_decoder="native", **kw))
    b = list(D.initialize_dataset(records, 8, jpeg_decoder="pillow", **kw))
    for (xa, ya), (xb, yb) in zip(a, b):
        np.testing.assert_array_equal(ya, yb)
        assert xa.shape == xb.shape
    c = list(D.initialize_dataset(records, 8, jpeg_decoder="native", jpeg_dct="islow", **kw))
    for (xc, _), (xb, _) in zip(c, b):
        np.testing.assert_array_equal(xc, xb)              # ISLOW: the pipeline's bytes == Pillow's
