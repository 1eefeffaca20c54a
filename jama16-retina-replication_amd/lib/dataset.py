"""Drop-in for the reference's lib/dataset.py (lib/dataset.py:1-59), no TF.

Same entry point and arguments:
    initialize_dataset(image_dir, batch_size, num_epochs=1, num_workers=1,
                       prefetch_buffer_size=None, shuffle_buffer_size=None,
                       image_data_format='channels_last', num_channels=3,
                       image_dim=[299, 299])
and the same element semantics:
  * files: every name in os.listdir(image_dir) ending in '.tfrecord', in
    os.listdir order (lib/dataset.py:5-8);
  * record -> (image, label): JPEG decode, f32(x) * f32(1/255)
    (tf.image.convert_image_dtype, :20-21), reshape to image_dim (:23;
    channels_first is a RESHAPE of the HWC buffer, App. C Q3), label int64 ->
    float32 [1] (:24-26);
  * shuffle(shuffle_buffer_size) if given (:50-51), repeat(num_epochs),
    batch(batch_size) keeping the partial last batch, prefetch (:53-57).
The returned Dataset is re-iterable: each `iter()` is a fresh
`sess.run(init_op)` (train.py:125-126,222).  Decoding runs on num_workers
threads (Pillow releases the GIL in its libjpeg decoder); prefetch runs the
pipeline on a background thread.

Extras (keyword-only, default off): `seed` for a reproducible shuffle (the
reference's is unseeded, App. C Q4), `decode_dtype='uint8'` to hand the
GPU the undecoded-scale bytes (libjr scales by 1/255 on device, 4x less
host->device traffic; values are bit-identical), and `shard=(rank, world)`
for data-parallel ranks: every rank walks the same (seeded) stream of record
handles and batches, and decodes only the batches b with b % world == rank
-- the per-record JPEG work is split across ranks, the batch composition is
that of the single-process stream.

JPEG decoding [TF-3P]: TF's decode_jpeg defaults to libjpeg-turbo's IFAST
IDCT.  The pipeline decodes natively (jr.jpeg, libjr_jpeg.so: IJG libjpeg 9
entropy decode + IDCT, libjpeg-turbo's upsampling and colour conversion
restated; outside the GIL, straight into the batch) with `jpeg_dct='ifast'`
(TF's default; 'islow' selectable), and falls back to Pillow (libjpeg-turbo,
ISLOW) when that library is not built (`jpeg_decoder='pillow'` forces it).
With ISLOW the native bytes equal Pillow's (tests/test_data_pipeline.py);
IFAST equals TF's decode to the extent IJG 9's AAN IDCT equals turbo's --
no turbo IFAST decoder is importable here, so that last step is unpinned.
"""
from __future__ import annotations

import collections
import io
import os
import queue
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Iterator, List, Optional, Tuple

import numpy as np

try:
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None

from jr import jpeg as native_jpeg
from jr import tfrecord

_SCALE = np.float32(1.0 / 255.0)


def _tfrecord_files_from_folder(folder: str, ext: str = ".tfrecord") -> List[str]:
    """lib/dataset.py:5-8: os.listdir order, filtered by extension."""
    return [os.path.join(folder, n) for n in os.listdir(folder) if n.endswith(ext)]


def decode_jpeg(data: bytes) -> np.ndarray:
    """tf.image.decode_jpeg(channels=0): HWC uint8 with the file's channels."""
    if Image is None:
        raise RuntimeError("Pillow is required to decode JPEG records")
    with Image.open(io.BytesIO(data)) as im:
        im.load()
        return np.asarray(im, dtype=np.uint8)


def _decode_one(data, jpeg_decoder: Optional[str] = None, jpeg_dct: str = "ifast") -> np.ndarray:
    """decode_jpeg by the pipeline's decoder (native when built, else Pillow)."""
    if jpeg_decoder is None:
        jpeg_decoder = "native" if native_jpeg.available() else "pillow"
    return native_jpeg.decode(data, jpeg_dct) if jpeg_decoder == "native" else decode_jpeg(data)


def _parse_example(record: bytes, image_dim, decode_dtype: str, jpeg_decoder: Optional[str] = None,
                   jpeg_dct: str = "ifast") -> Tuple[np.ndarray, np.ndarray]:
    """lib/dataset.py:11-28."""
    ex = tfrecord.decode_example(record)
    for key in ("image/encoded", "image/format", "image/class/label", "image/height", "image/width"):
        if key not in ex or len(ex[key]) != 1:
            raise ValueError(f"record is missing FixedLenFeature {key!r}")
    img = _decode_one(ex["image/encoded"][0], jpeg_decoder, jpeg_dct)
    if img.size != int(np.prod(image_dim)):
        raise ValueError(f"cannot reshape image of {img.size} values into {list(image_dim)}")
    img = img.reshape(image_dim)                 # reshape, not transpose (App. C Q3)
    if decode_dtype == "float32":
        img = img.astype(np.float32) * _SCALE    # convert_image_dtype: f32(x) * f32(1/255)
    label = np.array([ex["image/class/label"][0]], dtype=np.int64).astype(np.float32)
    return img, label


class Dataset:
    """Batched (images, labels) stream; iterate once per epoch group."""

    def __init__(self, files: List[str], batch_size: int, num_epochs: int, num_workers: int,
                 prefetch_buffer_size: Optional[int], shuffle_buffer_size: Optional[int],
                 image_dim: List[int], seed: Optional[int], decode_dtype: str,
                 shard: Optional[Tuple[int, int]] = None, jpeg_decoder: Optional[str] = None,
                 jpeg_dct: str = "ifast"):
        if batch_size <= 0:
            raise ValueError("batch_size must be positive")
        rank, world = shard or (0, 1)
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"bad shard {shard!r}: need 0 <= rank < world")
        self.shard = (int(rank), int(world))
        if jpeg_decoder is None:
            jpeg_decoder = "native" if native_jpeg.available() else "pillow"
        if jpeg_decoder not in ("native", "pillow") or jpeg_dct not in native_jpeg.DCT:
            raise ValueError("jpeg_decoder: 'native' or 'pillow'; jpeg_dct: 'ifast' or 'islow'")
        if jpeg_decoder == "native" and not native_jpeg.available():
            raise RuntimeError("jpeg_decoder='native' needs libjr_jpeg.so (csrc Makefile)")
        self.jpeg_decoder, self.jpeg_dct = jpeg_decoder, jpeg_dct
        self.files = files
        self.batch_size = int(batch_size)
        self.num_epochs = num_epochs
        self.num_workers = max(1, int(num_workers))
        self.prefetch_buffer_size = prefetch_buffer_size
        self.shuffle_buffer_size = shuffle_buffer_size
        self.image_dim = list(image_dim)
        self.decode_dtype = decode_dtype
        self._seed = seed
        self._rng = np.random.default_rng(seed)
        self._iteration = 0

    # ------------------------------------------------------------- stages
    def _items(self) -> Iterator[Tuple["tfrecord.RecordFile", int]]:
        """TFRecordDataset over the files in order: (file, record index) pairs.
        Each file is mmap'd and indexed natively (jr_tfrecord_index) and its
        Example features located in one call (jr_example_parse_image), so the
        per-record host work is only the JPEG decode on the worker threads."""
        for path in self.files:
            f = tfrecord.RecordFile(path)
            for i in range(f.num_records):
                yield f, i
            f.raise_if_damaged()               # DataLossError where tf.data would raise it

    def _shuffled(self, it):
        """tf.data shuffle: fill a buffer, emit a uniformly random element and
        refill its slot from the input; drain randomly at the end.  Applied to
        (file, record) handles before the map: the map is elementwise, so the
        emitted order is that of shuffling the decoded elements."""
        n = self.shuffle_buffer_size
        if n is None:
            yield from it
            return
        rng = self._iter_rng
        buf = []
        for x in it:
            if len(buf) < n:
                buf.append(x)
                continue
            i = int(rng.integers(len(buf)))
            out, buf[i] = buf[i], x
            yield out
        while buf:
            i = int(rng.integers(len(buf)))
            buf[i], buf[-1] = buf[-1], buf[i]
            yield buf.pop()

    def _all_item_batches(self) -> Iterator[list]:
        """repeat(num_epochs) then batch(batch_size), partial last batch kept."""
        epochs = self.num_epochs
        e = 0
        cur = []
        while epochs is None or epochs < 0 or e < epochs:
            any_elem = False
            for it in self._shuffled(self._items()):
                any_elem = True
                cur.append(it)
                if len(cur) == self.batch_size:
                    yield cur
                    cur = []
            e += 1
            if not any_elem:
                break
        if cur:
            yield cur

    def _item_batches(self) -> Iterator[list]:
        """This rank's batches (shard): handles only, before any decode."""
        rank, world = self.shard
        for b, items in enumerate(self._all_item_batches()):
            if b % world == rank:
                yield items

    def _decode(self, data: bytes, dst: Optional[np.ndarray]) -> np.ndarray:
        """One JPEG: natively (straight into dst when it is a uint8 row of the
        right size) or by Pillow."""
        if self.jpeg_decoder == "native":
            h, w, c = native_jpeg.header(data)
            if dst is not None and dst.dtype == np.uint8 and dst.size == h * w * c:
                return native_jpeg.decode(data, self.jpeg_dct, dst.reshape(-1)).reshape(h, w, c)
            return native_jpeg.decode(data, self.jpeg_dct)
        return decode_jpeg(data)

    def _decode_rows(self, items, rows, out) -> None:
        """map(_parse_example) for rows [rows) of one batch, written in place."""
        for r in rows:
            f, i = items[r]
            f.check(i)                                # FixedLenFeature checks (lib/dataset.py:12-16)
            img = self._decode(f.encoded(i), out[r] if self.decode_dtype == "uint8" else None)
            if img.size != out[r].size:
                raise ValueError(f"cannot reshape image of {img.size} values into {self.image_dim}")
            if img.base is not None and np.shares_memory(img, out[r]):
                continue                              # decoded in place (uint8)
            img = img.reshape(self.image_dim)        # reshape, not transpose (App. C Q3)
            if self.decode_dtype == "float32":
                np.multiply(img, _SCALE, out=out[r])  # convert_image_dtype: f32(x) * f32(1/255)
            else:
                out[r] = img

    def _submit(self, pool: ThreadPoolExecutor, items):
        n = len(items)
        out = np.empty([n] + self.image_dim, np.uint8 if self.decode_dtype == "uint8" else np.float32)
        labels = np.array([f.label[i] for f, i in items], np.int64).astype(np.float32).reshape(n, 1)
        chunk = max(1, -(-n // (2 * self.num_workers)))
        futs = [pool.submit(self._decode_rows, items, range(a, min(n, a + chunk)), out)
                for a in range(0, n, chunk)]
        return out, labels, futs

    def _batches(self) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
        depth = 2                                   # batches decoding ahead of the consumer
        with ThreadPoolExecutor(self.num_workers) as pool:
            inflight: "collections.deque" = collections.deque()
            batches, err = self._item_batches(), None
            try:
                while True:
                    try:
                        items = next(batches)
                    except StopIteration:
                        break
                    except Exception as e:              # damaged file: deliver what came before it
                        err = e
                        break
                    inflight.append(self._submit(pool, items))
                    if len(inflight) > depth:
                        yield _collect(inflight.popleft())
                while inflight:
                    yield _collect(inflight.popleft())
                if err is not None:
                    raise err
            finally:
                for _, _, futs in inflight:
                    for fu in futs:
                        fu.cancel()

    def __iter__(self):
        # seeded: iteration k shuffles with PCG64(seed, k) (tf.data's
        # reshuffle_each_iteration with a seed), so ranks that stop an epoch
        # early at different stream positions still agree on the next one;
        # unseeded: one process-wide stream, as the reference's
        self._iter_rng = (np.random.default_rng([self._seed, self._iteration]) if self._seed is not None
                          else self._rng)
        self._iteration += 1
        gen = self._batches()
        if not self.prefetch_buffer_size:
            return gen
        return _Prefetch(gen, max(1, int(self.prefetch_buffer_size) // self.batch_size + 1))

    def num_batches(self) -> int:
        """Batches of one pass over the whole (unsharded) stream."""
        n = self.num_records() * max(1, self.num_epochs or 1)
        return -(-n // self.batch_size)

    def num_records(self) -> int:
        n = 0
        for path in self.files:
            f = tfrecord.RecordFile(path, parse=False)
            f.raise_if_damaged()
            n += f.num_records
        return n


def _collect(entry):
    out, labels, futs = entry
    for fu in futs:
        fu.result()                                 # first failing row raises, in order
    return out, labels


class _Prefetch:
    """prefetch(): run the pipeline ahead on a background thread.

    close() (also on garbage collection, and implied by reaching the end)
    stops the thread at its next hand-off and closes the pipeline generator
    on that thread, so its decode pool and mmap'd files are released when a
    consumer stops early (a capped epoch, a `break`)."""

    _END = object()

    def __init__(self, gen, depth: int):
        self._q: "queue.Queue" = queue.Queue(maxsize=depth)
        self._err = None
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, args=(gen,), daemon=True)
        self._t.start()

    def _put(self, item) -> bool:
        while not self._stop.is_set():
            try:
                self._q.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _run(self, gen):
        try:
            for item in gen:
                if not self._put(item):
                    break
        except BaseException as e:  # surfaced to the consumer
            self._err = e
        finally:
            gen.close()             # runs the pipeline's finally: decode pool shutdown
        self._put(self._END)

    def __iter__(self):
        return self

    def __next__(self):
        if self._stop.is_set():
            raise StopIteration
        item = self._q.get()
        if item is self._END:
            self._stop.set()
            if self._err is not None:
                raise self._err
            raise StopIteration
        return item

    def close(self):
        self._stop.set()
        try:                        # unblock a producer waiting on a full queue
            while True:
                self._q.get_nowait()
        except queue.Empty:
            pass

    def join(self, timeout=None):
        self._t.join(timeout)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def initialize_dataset(image_dir, batch_size, num_epochs=1,
                       num_workers=1, prefetch_buffer_size=None,
                       shuffle_buffer_size=None,
                       image_data_format='channels_last',
                       num_channels=3, image_dim=[299, 299], *,
                       seed=None, decode_dtype="float32", shard=None, jpeg_decoder=None, jpeg_dct="ifast"):
    """lib/dataset.py:31-59 (same arguments, same order, same defaults)."""
    files = _tfrecord_files_from_folder(image_dir)
    if image_data_format == 'channels_first':
        dim = [num_channels, image_dim[0], image_dim[1]]
    elif image_data_format == 'channels_last':
        dim = [image_dim[0], image_dim[1], num_channels]
    else:
        raise TypeError('invalid image date format setting')
    if decode_dtype not in ("float32", "uint8"):
        raise ValueError("decode_dtype must be 'float32' or 'uint8'")
    return Dataset(files, batch_size, num_epochs, num_workers, prefetch_buffer_size,
                   shuffle_buffer_size, dim, seed, decode_dtype, shard, jpeg_decoder, jpeg_dct)


def close_iterator(it) -> None:
    """Release an iterator of a Dataset (prefetch thread or generator)."""
    close = getattr(it, "close", None)
    if close is not None:
        close()
