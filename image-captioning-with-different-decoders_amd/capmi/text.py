"""Caption tokenizer: the reference numericalizes captions with nltk.tokenize.word_tokenize on the
lower-cased text (dataset.py:45-51, vocabulary.py:42-46). nltk (and its punkt model) is absent
here, so `word_tokenize` uses nltk when importable and otherwise this restatement of nltk's
Treebank word tokenizer rules (starting quotes, punctuation, brackets, double dashes, ending
quotes and clitics, the contraction splits), applied to the whole caption as one sentence.
Parity with nltk is unpinned (no nltk outputs are available); on plain COCO captions (words,
commas, a final period) the rules reduce to whitespace splitting with punctuation split off.
"""
import re

_STARTING_QUOTES = [(re.compile(r'^\"'), r'``'), (re.compile(r'(``)'), r' \1 '),
                    (re.compile(r"([ \(\[{<])(\"|\'{2})"), r'\1 `` ')]
_PUNCTUATION = [
    (re.compile(r'([^\.])(\.)([\]\)}>"\']*)\s*$'), r'\1 \2 \3 '),
    (re.compile(r'([:,])([^\d])'), r' \1 \2'),
    (re.compile(r'([:,])$'), r' \1 '),
    (re.compile(r'\.\.\.'), r' ... '),
    (re.compile(r'[;@#$%&]'), r' \g<0> '),
    (re.compile(r'[?!]'), r' \g<0> '),
    (re.compile(r"([^'])' "), r"\1 ' "),
]
_PARENS = (re.compile(r'[\]\[\(\)\{\}\<\>]'), r' \g<0> ')
_DOUBLE_DASHES = (re.compile(r'--'), r' -- ')
_ENDING_QUOTES = [(re.compile(r'"'), " '' "), (re.compile(r"(\S)(\'\')"), r'\1 \2 '),
                  (re.compile(r"([^' ])('[sS]|'[mM]|'[dD]|') "), r'\1 \2 '),
                  (re.compile(r"([^' ])('ll|'LL|'re|'RE|'ve|'VE|n't|N'T) "), r'\1 \2 ')]
_CONTRACTIONS = [re.compile(p, re.I) for p in (
    r'\b(can)(not)\b', r"\b(d)('ye)\b", r'\b(gim)(me)\b', r'\b(gon)(na)\b', r'\b(got)(ta)\b',
    r'\b(lem)(me)\b', r"\b(more)('n)\b", r'\b(wan)(na)(?=\s)', r"('t)(is)\b", r"('t)(was)\b")]


def _treebank(text):
    for rx, sub in _STARTING_QUOTES:
        text = rx.sub(sub, text)
    for rx, sub in _PUNCTUATION:
        text = rx.sub(sub, text)
    text = _PARENS[0].sub(_PARENS[1], text)
    text = _DOUBLE_DASHES[0].sub(_DOUBLE_DASHES[1], text)
    text = ' ' + text + ' '
    for rx, sub in _ENDING_QUOTES:
        text = rx.sub(sub, text)
    for rx in _CONTRACTIONS:
        text = rx.sub(r' \1 \2 ', text)
    return text.split()


def word_tokenize(text):
    try:
        import nltk
        return nltk.tokenize.word_tokenize(text)
    except (ImportError, LookupError):  # no nltk, or no punkt model
        return _treebank(text)
