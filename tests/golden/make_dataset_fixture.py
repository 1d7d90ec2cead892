"""Expected parse of ASME's on-disk dataset format, produced by the READ-ONLY reference's
own readers on the example dataset its tests hold (copied as data to tests/golden/example_dataset/).

Build-container only (imports /root/reference).  Writes tests/golden/example_dataset_expected.json:
  sessions: every session of example.csv (+ the ratio split's train csv) tokenized with the vocabulary, read
            through CsvDatasetIndex / CsvDatasetReader / ItemSessionParser (data/base/reader.py,
            data/datasets/sequence.py) and the Tokenizer (core/tokenization/tokenizer.py);
  positions: (session, target_pos) pairs of the loo / nextitem indices read with SequencePositionIndex
            (data/datasets/index.py), and the (input, target) each yields after SequencePositionDataset's
            truncation to [:pos+1] (data/datasets/sequence_position.py:50-58) and TargetExtractorProcessor
            (data/datasets/processors/target_extractor.py:41-70).

    python tests/golden/make_dataset_fixture.py
"""
import json
import os
import sys
from pathlib import Path

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _ref_stubs as S  # noqa: E402

S.install()

from asme.core.tokenization.tokenizer import Tokenizer  # noqa: E402
from asme.core.tokenization.vocabulary import CSVVocabularyReaderWriter  # noqa: E402
from asme.data.base.reader import CsvDatasetIndex, CsvDatasetReader  # noqa: E402
from asme.data.datasets.index import SequencePositionIndex  # noqa: E402
from asme.data.datasets.sequence import ItemSessionParser, MetaInformation, PlainSequenceDataset  # noqa: E402

D = Path(HERE) / "example_dataset"


def tokenizer(path):
    with open(path) as f:
        return Tokenizer(CSVVocabularyReaderWriter().read(f), pad_token="<PAD>", mask_token="<MASK>",
                         unk_token="<UNK>")


def sessions(csv_path, idx_path, tok):
    with open(csv_path) as f:
        header = f.readline().rstrip("\n").split("\t")
    parser = ItemSessionParser({h: i for i, h in enumerate(header)},
                               [MetaInformation("item", "str", column_name="item_id", is_sequence=True)], "\t")
    ds = PlainSequenceDataset(CsvDatasetReader(Path(csv_path), CsvDatasetIndex(Path(idx_path))), parser)
    return [[int(t) for t in tok.convert_tokens_to_ids(ds[i]["item"])] for i in range(len(ds))]


def positions(idx_path, sess):
    index = SequencePositionIndex(Path(idx_path))
    out = []
    for i in range(len(index)):
        s, p = index[i]
        seq = sess[s][:p + 1]
        out.append({"session": int(s), "pos": int(p), "input": seq[:-1], "target": seq[-1]})
    return out


def main():
    tok = tokenizer(D / "example.vocabulary.item_id.txt")
    full = sessions(D / "example.csv", D / "example.session.idx", tok)
    tok_r = tokenizer(D / "ratio" / "example.vocabulary.item_id.txt")
    train = sessions(D / "ratio" / "example.train.csv", D / "ratio" / "example.train.session.idx", tok_r)
    out = {
        "sessions": full,
        "ratio_train_sessions": train,
        "loo": {k: positions(D / "loo" / f"example.{k}.loo.idx", full) for k in ("train", "validation", "test")},
        "nextitem": positions(D / "loo" / "example.nextitem.idx", full),
        "ratio_train_nextitem": positions(D / "ratio" / "example.train.nextitem.idx", train),
    }
    with open(os.path.join(HERE, "example_dataset_expected.json"), "w") as f:
        json.dump(out, f, indent=1)
    print({k: (len(v) if isinstance(v, list) else {kk: len(vv) for kk, vv in v.items()}) for k, v in out.items()})


if __name__ == "__main__":
    main()
