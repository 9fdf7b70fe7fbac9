"""Data feed: samplers, per-epoch order, collate, dataset readers.

Batch lists, epoch orders and the collate output are compared EXACTLY with golden vectors
produced by the reference's own build_batch_sampler / SequenceIterFactory / common_collate_fn
(tests/golden/make_data_feed_golden.py).  File readers round-trip through the writers here
(Kaldi ark, PCM WAV, npy); the reference's fileio tests (test/espnet2/fileio) use the same
round-trip style.  CPU only.
"""
import json
import os
import struct

import numpy as np
import pytest
import torch

from espnet_slurp_amd.fileio.kaldi_ark import KaldiArkScpReader, read_ark, write_ark
from espnet_slurp_amd.fileio.npy_scp import NpyScpReader
from espnet_slurp_amd.fileio.read_text import load_num_sequence_text, read_2column_text
from espnet_slurp_amd.fileio.sound_scp import SoundScpReader, read_wav, write_wav
from espnet_slurp_amd.iterators.sequence_iter_factory import SequenceIterFactory, shard_batches
from espnet_slurp_amd.samplers import build_batch_sampler
from espnet_slurp_amd.train.collate_fn import CommonCollateFn, common_collate_fn
from espnet_slurp_amd.train.dataset import ESPnetDataset

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "data_feed.json")))


def _write(path, tab):
    with open(path, "w") as f:
        for k, v in tab.items():
            f.write(k + " " + (",".join(map(str, v)) if isinstance(v, list) else str(v)) + "\n")


@pytest.fixture(scope="module")
def shape_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("shapes")
    paths = {}
    for name in ("speech_shape", "text_shape", "utt2category"):
        paths[name] = str(d / name)
        _write(paths[name], GOLD[name])
    return paths


@pytest.mark.parametrize("case", range(len(GOLD["cases"])))
def test_sampler_matches_reference(shape_dir, case):
    c = GOLD["cases"][case]
    kw = dict(c["kwargs"])
    if kw.get("utt2category_file"):
        kw["utt2category_file"] = shape_dir["utt2category"]
    s = build_batch_sampler(shape_files=[shape_dir["speech_shape"], shape_dir["text_shape"]], **kw)
    assert [list(b) for b in s] == c["batches"]


def test_sampler_errors(shape_dir):
    sp = [shape_dir["speech_shape"]]
    with pytest.raises(ValueError):
        build_batch_sampler("bogus", 1, 1, sp)
    with pytest.raises(ValueError):
        build_batch_sampler("numel", 1, 100, [])
    with pytest.raises(ValueError):
        build_batch_sampler("folded", 4, 1, sp, fold_lengths=[1, 2])
    with pytest.raises(ValueError):
        build_batch_sampler("numel", 1, 100, sp, sort_batch="sideways")


@pytest.mark.parametrize("n_it", ["None", "3", "40"])
def test_epoch_order_matches_reference(n_it):
    e = GOLD["epochs"]
    batches = [tuple(b) for b in e["batches"]]
    f = SequenceIterFactory(dataset=None, batches=batches, num_iters_per_epoch=None if n_it == "None" else int(n_it),
                            seed=e["seed"], shuffle=True)
    for ep, want in e["orders"][n_it].items():
        assert [list(b) for b in f.epoch_batches(int(ep))] == want


def test_shard_batches():
    b = [("a", "b", "c", "d", "e"), ("f", "g")]
    assert shard_batches(b, 0, 2) == [("a", "c", "e"), ("f",)]
    assert shard_batches(b, 1, 2) == [("b", "d"), ("g",)]
    with pytest.raises(RuntimeError):
        shard_batches(b, 0, 3)


def test_collate_matches_reference():
    g = GOLD["collate"]
    data = [(u, {k: np.array(v, dtype=np.float32 if k == "speech" else np.int64) for k, v in d.items()})
            for u, d in g["inputs"].items()]
    ids, out = CommonCollateFn(float_pad_value=0.0, int_pad_value=-1)(data)
    assert ids == g["ids"]
    assert set(out) == set(g["out"])
    for k, v in g["out"].items():
        assert out[k].tolist() == v, k
    assert out["text"].dtype == torch.int64 and out["speech_lengths"].dtype == torch.int64


@pytest.mark.parametrize("fpad, ipad, not_seq", [(0.0, -1, ()), (3.0, 2, ("a",)), (np.inf, 100, ("a", "b"))])
def test_collate_padding_rules(fpad, ipad, not_seq):
    rng = np.random.RandomState(0)
    data = [("id", dict(a=rng.randn(3, 5), b=rng.randint(0, 9, 4))),
            ("id2", dict(a=rng.randn(2, 5), b=rng.randint(0, 9, 3)))]
    ids, t = common_collate_fn(data, float_pad_value=fpad, int_pad_value=ipad, not_sequence=not_seq)
    want_a = np.stack([data[0][1]["a"], np.pad(data[1][1]["a"], [(0, 1), (0, 0)], constant_values=fpad)])
    want_b = np.stack([data[0][1]["b"], np.pad(data[1][1]["b"], [(0, 1)], constant_values=ipad)])
    np.testing.assert_array_equal(t["a"].numpy(), want_a)
    np.testing.assert_array_equal(t["b"].numpy(), want_b)
    assert ("a_lengths" in t) == ("a" not in not_seq)
    assert ("b_lengths" in t) == ("b" not in not_seq)
    with pytest.raises(AssertionError):
        common_collate_fn([("x", {"a_lengths": np.zeros(2)})])


def test_read_text_tables(tmp_path):
    p = tmp_path / "t"
    p.write_text("k1 1,2,3\nk2 4\nk3\n")
    assert read_2column_text(p) == {"k1": "1,2,3", "k2": "4", "k3": ""}
    p2 = tmp_path / "t2"
    p2.write_text("k1 1 2 3\nk2 4\n")
    assert load_num_sequence_text(p2, "text_int") == {"k1": [1, 2, 3], "k2": [4]}
    p.write_text("a 1\na 2\n")
    with pytest.raises(RuntimeError):
        read_2column_text(p)
    with pytest.raises(ValueError):
        load_num_sequence_text(p2, "bogus")


def test_kaldi_ark_roundtrip(tmp_path):
    rng = np.random.RandomState(1)
    items = {"u1": rng.randn(7, 80).astype(np.float32), "u2": rng.randn(3, 80).astype(np.float64),
             "u3": rng.randn(5).astype(np.float32)}
    ark = str(tmp_path / "feats.ark")
    scp = write_ark(ark, items)
    _write(str(tmp_path / "feats.scp"), scp)
    r = KaldiArkScpReader(str(tmp_path / "feats.scp"))
    for k, v in items.items():
        np.testing.assert_array_equal(r[k], v)
        assert r[k].dtype == v.dtype
    assert [k for k, _ in read_ark(ark)] == list(items)
    with open(str(tmp_path / "bad.ark"), "wb") as f:
        f.write(b"k \0BCM " + b"\0" * 32)
    _write(str(tmp_path / "bad.scp"), {"k": f"{tmp_path}/bad.ark:2"})
    with pytest.raises(NotImplementedError):
        KaldiArkScpReader(str(tmp_path / "bad.scp"))["k"]


def test_wav_reader(tmp_path):
    rng = np.random.RandomState(2)
    pcm = rng.randint(-32768, 32768, 1000).astype(np.int16)
    write_wav(str(tmp_path / "a.wav"), pcm, 16000)
    x, rate = read_wav(str(tmp_path / "a.wav"), normalize=True)
    assert rate == 16000 and x.dtype == np.float64
    np.testing.assert_array_equal(x, pcm / 32768.0)
    raw, _ = read_wav(str(tmp_path / "a.wav"), normalize=False)
    np.testing.assert_array_equal(raw, pcm)
    st = rng.randint(-32768, 32768, (50, 2)).astype(np.int16)
    write_wav(str(tmp_path / "s.wav"), st, 8000)
    y, _ = read_wav(str(tmp_path / "s.wav"))
    assert y.shape == (50, 2)
    # 24-bit PCM written by hand
    v = np.array([-(1 << 23), -1, 0, 1, (1 << 23) - 1], dtype=np.int32)
    data = b"".join(struct.pack("<i", int(t))[:3] for t in v)
    hdr = (b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE" + b"fmt " +
           struct.pack("<IHHIIHH", 16, 1, 1, 16000, 48000, 3, 24) + b"data" + struct.pack("<I", len(data)))
    (tmp_path / "p24.wav").write_bytes(hdr + data)
    z, _ = read_wav(str(tmp_path / "p24.wav"))
    np.testing.assert_array_equal(z, v / float(1 << 23))
    (tmp_path / "x.flac").write_bytes(b"fLaC" + b"\0" * 40)
    with pytest.raises(NotImplementedError, match="audio_format wav"):  # actionable: SLURP dumps FLAC by default
        read_wav(str(tmp_path / "x.flac"))


def test_dataset_and_loader_end_to_end(tmp_path):
    """wav.scp + text_int -> ESPnetDataset -> sampler -> collate: the batch dict the model
    consumes (speech float32 padded 0.0, text int64 padded -1, *_lengths)."""
    rng = np.random.RandomState(4)
    wav, txt, shp = {}, {}, {}
    for i, n in enumerate([1600, 800, 1200, 400]):
        k = f"u{i}"
        write_wav(str(tmp_path / f"{k}.wav"), rng.randint(-3000, 3000, n).astype(np.int16), 16000)
        wav[k] = str(tmp_path / f"{k}.wav")
        txt[k] = " ".join(str(t) for t in rng.randint(2, 30, 3 + i))
        shp[k] = [n]
    _write(str(tmp_path / "wav.scp"), wav)
    _write(str(tmp_path / "text"), txt)
    _write(str(tmp_path / "speech_shape"), shp)
    ds = ESPnetDataset([(str(tmp_path / "wav.scp"), "speech", "sound"), (str(tmp_path / "text"), "text", "text_int")])
    uid, d = ds["u2"]
    assert d["speech"].dtype == np.float32 and d["text"].dtype == np.int64 and d["speech"].shape == (1200,)
    s = build_batch_sampler("numel", 1, 3000, [str(tmp_path / "speech_shape")])
    f = SequenceIterFactory(ds, list(s), seed=0, shuffle=True, collate_fn=CommonCollateFn(0.0, -1))
    seen = []
    for ids, b in f.build_iter(1):
        assert b["speech"].shape[0] == len(ids) and b["speech"].dtype == torch.float32
        assert int(b["speech_lengths"].max()) == b["speech"].shape[1]
        assert (b["text"] == -1).sum() == sum(b["text_lengths"].max() - b["text_lengths"])
        seen += ids
    assert sorted(seen) == sorted(wav)
    with pytest.raises(ValueError):
        ESPnetDataset([(str(tmp_path / "wav.scp"), "speech", "hdf5")])
    with pytest.raises(RuntimeError):
        ESPnetDataset([(str(tmp_path / "wav.scp"), "x", "sound"), (str(tmp_path / "text"), "x", "text_int")])
    np.save(str(tmp_path / "f.npy"), rng.randn(5, 80).astype(np.float64))
    _write(str(tmp_path / "npy.scp"), {"u0": str(tmp_path / "f.npy")})
    ds2 = ESPnetDataset([(str(tmp_path / "npy.scp"), "speech", "npy")])
    assert ds2["u0"][1]["speech"].dtype == np.float32
    assert len(NpyScpReader(str(tmp_path / "npy.scp"))) == 1
    assert SoundScpReader(str(tmp_path / "wav.scp"))["u0"][0] == 16000
