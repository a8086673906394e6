"""Native WordPiece tokenizer (csrc/runtime/tokenizer.cpp) against an
independent implementation: HF ``tokenizers.BertWordPieceTokenizer`` (Rust
BertNormalizer + BertPreTokenizer + WordPiece) on a vocab file generated here.
No real vocab ships offline; the contract under test is text -> ids for a
given vocab (reference embed contract providers.py:36-57)."""
import random

import pytest

tokenizers = pytest.importorskip("tokenizers")

from lazzaro_amd.core.embedders import Tokenizer  # noqa: E402

SENTENCES = [
    "Hello World!", "I am running, playing; unbelievable.", "Café naïve résumé Ångström",
    "我爱北京 hello", "—“quoted”— text", "tab\there\nnewline  spaces", "한국 hello", "x" * 150,
    "\x00ctrl\x07char​zw", "ﬁne ligature", "İstanbul", "ß straße", "Ⅻ roman", "emoji 😀 ok",
    "áb combining", "Ελληνικά Κείμενο", "Русский ТЕКСТ, да!", "x y z　w",
    "don't stop-believing... (really) [ok] {fine} <tag> a/b\\c", "ＦＵＬＬ width", "naïve­soft",
]

POOL = ([chr(c) for c in range(0x20, 0x7f)] + [chr(c) for c in range(0xa0, 0x180)] +
        [chr(c) for c in range(0x391, 0x3ca)] + [chr(c) for c in range(0x410, 0x450)] +
        list("我爱北京天安门한국어日本語") + ["́", "̈", "​", "—", "“", "、", "\t", "\n",
                                      " ", "😀", "ﬁ"])


def _vocab(tmp_path, corpus):
    hf_norm = tokenizers.normalizers.BertNormalizer(lowercase=True)
    pre = tokenizers.pre_tokenizers.BertPreTokenizer()
    words = set()
    for s in corpus:
        for w, _ in pre.pre_tokenize_str(hf_norm.normalize_str(s)):
            words.add(w)
    rng = random.Random(0)
    toks = set()
    for w in sorted(words):
        if rng.random() < 0.3:
            toks.add(w)  # whole word
        chars = list(w)
        toks.add(chars[0])
        toks.update("##" + c for c in chars[1:])
        if len(chars) > 3 and rng.random() < 0.5:
            toks.add("##" + "".join(chars[1:3]))
    vocab = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    vocab += sorted(t for t in toks if rng.random() < 0.92)  # some pieces missing -> [UNK] paths
    p = tmp_path / "vocab.txt"
    p.write_text("\n".join(vocab) + "\n", encoding="utf-8")
    return str(p)


def test_wordpiece_matches_hf_tokenizers(tmp_path):
    rng = random.Random(42)
    fuzz = ["".join(rng.choice(POOL) for _ in range(rng.randint(1, 40))) for _ in range(400)]
    corpus = SENTENCES + fuzz
    vf = _vocab(tmp_path, corpus)
    hf = tokenizers.BertWordPieceTokenizer(vf, lowercase=True)
    ours = Tokenizer(vf)
    for s in corpus:
        assert ours.encode(s, 512) == hf.encode(s).ids, repr(s)
    # batch form: same ids, [PAD] from the vocab, per-row lengths
    ids, lens = ours.encode_batch(corpus[:32], 512)
    for j, s in enumerate(corpus[:32]):
        want = hf.encode(s).ids
        assert int(lens[j]) == len(want) and ids[j, : len(want)].tolist() == want
        assert (ids[j, len(want):] == 0).all()


def test_truncation_keeps_cls_sep(tmp_path):
    vf = _vocab(tmp_path, SENTENCES)
    hf = tokenizers.BertWordPieceTokenizer(vf, lowercase=True)
    hf.enable_truncation(16)
    ours = Tokenizer(vf)
    for s in SENTENCES:
        assert ours.encode(s, 16) == hf.encode(s).ids, repr(s)
