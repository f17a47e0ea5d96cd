"""Tokenizer parity: native C++ featurizer == Python restatement == reference golden cases
(recorded from /root/reference/utils/data_utils.py under Python 3)."""
import json

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from dnn_page_vectors_amd.data import text as T
from dnn_page_vectors_amd.data.featurize import Featurizer, clean_str_native, generate_vocabulary

GOLD = "Statue of Liberty! NYC #1 tour, $25.00 (Mütze) a-b_c"


def test_clean_str_golden():
    assert T.clean_str(GOLD) == "statue of liberty  nyc #1 tour  $25.00  mütze  a b_c"
    assert clean_str_native(GOLD) == T.clean_str(GOLD)


def test_splits_golden():
    assert T.split_features(GOLD, "word") == ["statue", "of", "liberty", "", "nyc", "#1", "tour", "", "$25.00", "",
                                              "mütze", "", "a", "b_c"]
    assert T.split_features(GOLD, "word", 3) == ["statue", "of", "liberty"]
    assert T.split_features(GOLD, "char", 12) == list("statue of li")
    assert T.split_features(GOLD, "ngram", 6) == ["sta", "tat", "atu", "tue", "ue ", "e o"]


def test_pad_and_vocab_order():
    assert T.pad_tokens(["a"], 3) == ["a", "<PAD/>", "<PAD/>"]
    assert T.build_vocab_counts([["b", "a", "b"], ["c", "a", "b"]]) == ["b", "a", "c"]
    v = T.Vocab(["x", "y"])
    assert v.itos[:3] == ["<PAD/>", "<UNK/>", " "] and v.lookup("zzz") == v.unk_id == 1 and v.pad_id == 0


def test_empty_and_short_texts():
    assert T.split_features("", "word") == [""]          # ''.split(' ') == ['']
    assert T.split_features("ab", "ngram") == []
    assert T.split_features("!!!", "char") == []


@pytest.mark.parametrize("mode", ["word", "char", "ngram"])
def test_native_matches_python_vocab(mode):
    texts = [GOLD, "statue of liberty", "New York city", "", "a  b", "ÄÖÜ straße €5.00 #tag"]
    toks = [T.split_features(t, mode) for t in texts]
    vocab = T.Vocab(T.build_vocab_counts(toks))
    L = 17
    fz = Featurizer(mode, vocab=vocab, nthreads=2)
    got = fz(texts, L)
    want = np.array(T.featurize_py(texts, mode, L, vocab=vocab), dtype=np.int32)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("mode", ["word", "char", "ngram"])
def test_native_matches_python_hash(mode):
    texts = [GOLD, "statue of liberty", "ümlaut ß €", "x"]
    fz = Featurizer(mode, hash_size=1000, nthreads=3)
    got = fz(texts, 25)
    want = np.array(T.featurize_py(texts, mode, 25, hash_size=1000), dtype=np.int32)
    np.testing.assert_array_equal(got, want)
    assert got.min() >= 0 and got.max() < 1000


_ALPH = st.sampled_from(list("abcXYZ019 _-!.,#$€äöüßÄÖÜé\n\t()'\""))


@settings(max_examples=150, deadline=None)
@given(st.lists(st.text(alphabet=_ALPH, min_size=0, max_size=40), min_size=1, max_size=6),
       st.sampled_from(["word", "char", "ngram"]), st.integers(min_value=1, max_value=30))
def test_native_featurizer_fuzz(texts, mode, L):
    fz = Featurizer(mode, hash_size=4096, nthreads=2)
    got = fz(texts, L)
    want = np.array(T.featurize_py(texts, mode, L, hash_size=4096), dtype=np.int32)
    np.testing.assert_array_equal(got, want)
    for t in texts:
        assert clean_str_native(t) == T.clean_str(t)


def test_generate_vocabulary_skips_bad_rows(tmp_path):
    f = tmp_path / "train.txt"
    rows = [{"q": "statue", "doc_corr": "statue of liberty", "doc_incorr": ["a", "b", "c"]},
            {"q": "skip", "doc_corr": "zzz", "doc_incorr": ["only one"]}]
    f.write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    v = generate_vocabulary([str(f)], "word", 3)
    assert "statue" in v.stoi and "zzz" not in v.stoi
    # deterministic order: reserved, then by count desc
    assert v.itos[3] == "statue"


def test_html_normalizer():
    s = T.normalize_html_line("<b>Hello</b>   World&amp;Co...  Mütze!")
    assert "<b>" not in s and "  " not in s
    assert " . " in s and "mütze" in s


@settings(max_examples=100, deadline=None)
@given(st.lists(st.text(alphabet=st.sampled_from(list("abcXYZ019 _.#$€äöüßÄÖÜé\n\U0001F600\U00010400")),
                        min_size=0, max_size=40), min_size=1, max_size=5),
       st.integers(min_value=1, max_value=30))
def test_native_char_vocab_fuzz(texts, L):
    """char mode with an exact vocabulary: the native code-point table (BMP) and the string
    fallback (non-BMP code points, incl. a Deseret letter that lower-cases to another
    non-BMP code point) agree with the Python rules; ids of characters missing from the
    vocabulary are UNK; vocabulary edits after first use invalidate the table."""
    toks = [T.split_features(t, "char") for t in texts[:2]]  # later texts: OOV chars possible
    vocab = T.Vocab(T.build_vocab_counts(toks))
    fz = Featurizer("char", vocab=vocab, nthreads=2)
    got = fz(texts, L)
    want = np.array(T.featurize_py(texts, "char", L, vocab=vocab), dtype=np.int32)
    np.testing.assert_array_equal(got, want)
    fz._lib.pv_vocab_add(fz.handle(), "ü".encode(), 77)  # edit after the table was built
    got2 = fz(["über"], 4)
    assert got2[0, 0] == 77


# ---- HTML normalisation in the native featurizer (cfg.html_normalize) -----------------------
HTML_GOLD = [
    ("Hello &amp; <b>World</b>... Foo", "hello world . foo"),
    ("<p>Caf&eacute; &lt;b&gt;x&lt;/b&gt; &#39;q&#39; &#x41;</p>", "café x q a"),
    ("<script>var a = 1 < 2;</script>text", "var a 1 2 text"),
    ("a;lt;b ;amp; c", "ab c"),
    ("<!-- c -->x<?pi?>y<!DOCTYPE html>z", "xyz"),
    ("Ünïcödé   Straße  €5.00!!! ...", "ünïcödé straße €5 . 00 . "),
    ("&notit; &amp &ampx &#0; &#x110000; &#128;", " it x €"),
    ("<a href='x>y'>link</a> rest", "link rest"),
    ("5 < 6 and 7 > 3", "5 6 and 7 3"),
]


def test_html_normalize_native_golden():
    from dnn_page_vectors_amd.data.featurize import normalize_html_native

    for src, want in HTML_GOLD:
        assert T.normalize_html_line(src) == want, src
        assert normalize_html_native(src) == want, src


_WORDS = st.sampled_from(["page", "Straße", "NYC", "$25.00", "a-b_c", "x...y", "über", "Ω", "#1", "é", "12", "."])
_ENTS = st.sampled_from(["&amp;", "&lt;", "&gt;", "&quot;", "&#39;", "&nbsp;", "&eacute;", "&#x41;", "&#8364;",
                         "&copy", "&notin;", "&bogus;", "&", ";lt;", ";amp;"])
_TAGS = st.sampled_from(["<b>", "</b>", "<p class=\"x\">", "<br/>", "<a href='u?a=1&b=2'>", "</a>", "<!-- note -->",
                         "<img src=x.png alt=\"a > b\">", "</ p>", "<?php x ?>", "<!DOCTYPE html>", " < ", " > "])
_SEPS = st.sampled_from([" ", "  ", "\t", "\n", "", ", ", "!", "..."])


@st.composite
def _html_line(draw):
    parts = draw(st.lists(st.one_of(_WORDS, _ENTS, _TAGS, _SEPS), min_size=0, max_size=24))
    if draw(st.booleans()):
        parts.insert(draw(st.integers(0, len(parts))), "<script>if (a < b) { x = '&amp;'; }</script>")
    return "".join(parts)


@settings(max_examples=300, deadline=None)
@given(_html_line())
def test_html_normalize_native_fuzz(line):
    """The C++ normaliser equals data/text.py::normalize_html_line (Python's html.unescape +
    HTMLParser) on generated HTML fragments: tags with quoted / unquoted attributes, end tags,
    comments, declarations, processing instructions, named / numeric / legacy / unknown
    entities, script content, dot runs, tabs and newlines."""
    from dnn_page_vectors_amd.data.featurize import normalize_html_native

    assert normalize_html_native(line) == T.normalize_html_line(line)


@pytest.mark.parametrize("mode", ["word", "ngram", "char"])
def test_featurizer_html_mode_matches_python(mode):
    texts = [src for src, _ in HTML_GOLD] + ["plain text", ""]
    fz = Featurizer(mode, hash_size=1000, html=True)
    got = fz(texts, 24)
    want = np.array(T.featurize_py(texts, mode, 24, hash_size=1000, html=True), dtype=np.int32)
    np.testing.assert_array_equal(got, want)
    # and the flag matters: without it the markup is tokenised
    assert not np.array_equal(Featurizer(mode, hash_size=1000)(texts, 24), got)


def test_dataset_html_mode(tmp_path):
    from dnn_page_vectors_amd.data.dataset import JsonlPairDataset

    p = tmp_path / "d.jsonl"
    rows = [{"q": "caf&eacute; <b>menu</b>", "doc_corr": "<p>The Caf&eacute; &amp; bar...</p>",
             "doc_incorr": ["<i>x</i>", "y &lt; z", "<!-- c -->w"]}]
    p.write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    fz = Featurizer("word", hash_size=500, html=True)
    ds = JsonlPairDataset(str(p), fz, 6, 10, 3)
    q, d = ds.batch(np.array([0]))
    np.testing.assert_array_equal(q[0], T.featurize_py([rows[0]["q"]], "word", 6, hash_size=500, html=True)[0])
    want = T.featurize_py([rows[0]["doc_corr"]] + rows[0]["doc_incorr"], "word", 10, hash_size=500, html=True)
    np.testing.assert_array_equal(d[0], np.array(want, dtype=np.int32))
