"""Golden vectors for the data feed, generated in THIS container from the
reference's own samplers / iterator factory / collate (imported through refshim).  Output:
tests/golden/data_feed.json (the synthetic shape tables + the reference's batch lists) — data
only; nothing under /root/reference is copied.  Run:  python tests/golden/make_data_feed_golden.py
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden import refshim  # noqa: E402


def shape_tables(seed=0, n=53):
    rng = np.random.RandomState(seed)
    speech = {f"utt{i:03d}": [int(rng.randint(150, 1600)), 80] for i in range(n)}
    # a few equal lengths exercise the stable sort
    for i in range(0, n, 11):
        speech[f"utt{i:03d}"][0] = 700
    text = {k: [int(rng.randint(3, 41)), 600] for k in speech}
    cat = {k: ("A" if rng.rand() < 0.5 else "B") for k in speech}
    return speech, text, cat


def write_table(path, tab):
    with open(path, "w") as f:
        for k, v in tab.items():
            f.write(k + " " + (",".join(str(x) for x in v) if isinstance(v, list) else str(v)) + "\n")


CASES = [
    ("numel", dict(batch_bins=400000, min_batch_size=1)),
    ("numel", dict(batch_bins=400000, min_batch_size=4)),
    ("numel", dict(batch_bins=900000, sort_in_batch="ascending", sort_batch="descending")),
    ("numel", dict(batch_bins=500000, padding=False, drop_last=True)),
    ("numel", dict(batch_bins=250000, min_batch_size=3, drop_last=True)),
    ("length", dict(batch_bins=6000, min_batch_size=2)),
    ("length", dict(batch_bins=6000, padding=False, sort_batch="descending")),
    ("folded", dict(batch_size=12, fold_lengths=[800, 150])),
    ("folded", dict(batch_size=12, fold_lengths=[800, 150], min_batch_size=5, drop_last=True)),
    ("folded", dict(batch_size=8, fold_lengths=[500, 100], utt2category_file=True)),
    ("sorted", dict(batch_size=7)),
    ("sorted", dict(batch_size=7, sort_in_batch="ascending", drop_last=True)),
    ("unsorted", dict(batch_size=6)),
    ("unsorted", dict(batch_size=6, drop_last=True)),
]


def main():
    refshim.install()
    from espnet2.iterators.sequence_iter_factory import SequenceIterFactory
    from espnet2.samplers.build_batch_sampler import build_batch_sampler
    from espnet2.train.collate_fn import common_collate_fn

    speech, text, cat = shape_tables()
    out = {"speech_shape": speech, "text_shape": text, "utt2category": cat, "cases": []}
    with tempfile.TemporaryDirectory() as d:
        sp, tp, cp = (os.path.join(d, n) for n in ("speech_shape", "text_shape", "utt2category"))
        write_table(sp, speech)
        write_table(tp, text)
        write_table(cp, cat)
        for typ, kw in CASES:
            kw = dict(kw)
            if kw.get("utt2category_file"):
                kw["utt2category_file"] = cp
            args = dict(type=typ, batch_size=kw.pop("batch_size", 1), batch_bins=kw.pop("batch_bins", 1),
                        shape_files=[sp, tp], **kw)
            s = build_batch_sampler(**args)
            rec = {k: v for k, v in args.items() if k != "shape_files"}
            if rec.get("utt2category_file"):
                rec["utt2category_file"] = True
            out["cases"].append({"kwargs": rec, "batches": [list(b) for b in s]})
        # per-epoch order (shuffle + num_iters_per_epoch windows) over the first numel sampler
        batches = [list(b) for b in build_batch_sampler("numel", 1, 400000, [sp, tp])]
        ep = {}
        for n_it in (None, 3, 40):
            f = SequenceIterFactory(dataset=None, batches=batches, num_iters_per_epoch=n_it, seed=5, shuffle=True)
            ep[str(n_it)] = {str(e): [list(b) for b in f.build_iter(e).batch_sampler] for e in (1, 2, 3, 7)}
        out["epochs"] = {"batches": batches, "seed": 5, "orders": ep}
    # collate: padding / lengths of the reference function on fixed arrays
    rng = np.random.RandomState(3)
    data = [("a", dict(speech=rng.randn(5, 3).astype(np.float32), text=np.array([4, 5, 6]))),
            ("b", dict(speech=rng.randn(2, 3).astype(np.float32), text=np.array([7])))]
    ids, b = common_collate_fn(data, float_pad_value=0.0, int_pad_value=-1)
    out["collate"] = {"inputs": {u: {k: v.tolist() for k, v in d.items()} for u, d in data},
                      "ids": ids, "out": {k: v.tolist() for k, v in b.items()}}
    with open(os.path.join(HERE, "data_feed.json"), "w") as f:
        json.dump(out, f)
    print("wrote", os.path.join(HERE, "data_feed.json"), len(out["cases"]), "sampler cases")


if __name__ == "__main__":
    main()
