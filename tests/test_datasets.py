"""ASME's on-disk dataset format: the host readers against the parse the reference's own
readers produce on the example dataset its tests hold (tests/golden/make_dataset_fixture.py ->
tests/golden/example_dataset_expected.json), and the GPU position batches (asme_position_batch)."""
import json
import os

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
D = os.path.join(HERE, "golden", "example_dataset")
EXPECTED = json.load(open(os.path.join(HERE, "golden", "example_dataset_expected.json")))


def test_read_sessions_matches_reference_reader(asme):
    got = asme.datasets.read_sessions(os.path.join(D, "example.csv"), os.path.join(D, "example.session.idx"),
                                      os.path.join(D, "example.vocabulary.item_id.txt"))
    assert got == EXPECTED["sessions"]
    got = asme.datasets.read_sessions(os.path.join(D, "ratio", "example.train.csv"),
                                      os.path.join(D, "ratio", "example.train.session.idx"),
                                      os.path.join(D, "ratio", "example.vocabulary.item_id.txt"))
    assert got == EXPECTED["ratio_train_sessions"]


@pytest.mark.parametrize("name,path", [("train", "loo/example.train.loo.idx"),
                                       ("validation", "loo/example.validation.loo.idx"),
                                       ("test", "loo/example.test.loo.idx"),
                                       ("nextitem", "loo/example.nextitem.idx")])
def test_read_position_index_matches_reference(asme, name, path):
    pairs = asme.datasets.read_position_index(os.path.join(D, path))
    want = EXPECTED["loo"][name] if name != "nextitem" else EXPECTED["nextitem"]
    assert [tuple(map(int, p)) for p in pairs] == [(w["session"], w["pos"]) for w in want]


def test_vocabulary_reader(asme):
    v = asme.datasets.read_vocabulary(os.path.join(D, "example.vocabulary.item_id.txt"))
    assert v["<PAD>"] == 0 and v["<MASK>"] == 1 and v["<UNK>"] == 2 and len(v) == 13


@pytest.mark.gpu
@pytest.mark.parametrize("L", [2, 8])
@pytest.mark.parametrize("split", ["test", "nextitem"])
def test_position_batch_matches_reference(asme, dev, L, split):
    store = asme.datasets.load_session_store(os.path.join(D, "example.csv"), os.path.join(D, "example.session.idx"),
                                             os.path.join(D, "example.vocabulary.item_id.txt"), dev)
    path = "loo/example.test.loo.idx" if split == "test" else "loo/example.nextitem.idx"
    pairs = torch.from_numpy(asme.datasets.read_position_index(os.path.join(D, path)))
    items, lengths, target = asme.datasets.position_batch(store, pairs, L)
    assert int(asme.datasets.position_batch.last_error.item()) == 0
    want = EXPECTED["loo"]["test"] if split == "test" else EXPECTED["nextitem"]
    for i, w in enumerate(want):
        x = w["input"][-L:]
        assert items[i].tolist() == x + [0] * (L - len(x))
        assert int(lengths[i]) == len(x) and int(target[i]) == w["target"]
