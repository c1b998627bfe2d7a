"""Offline NLP for round-secret construction.

Reference: ``select_descriptive_words`` (``src/utils.py:81-104``) tokenises with
``nltk.word_tokenize``, POS-tags with nltk's averaged perceptron, keeps alphabetic tokens
tagged JJ/JJR/JJS/RB/RBR/RBS/NN/NNS, scores each by the L2 distance of its word vector from
the mean vector of the kept words (``semantic_distance``, ``src/utils.py:74-79``; 0 if OOV),
multiplies by a single-document TF-IDF weight (≡1.0) and masks the top
``num_words``.  nltk and its corpora are not available offline (and never will be on the GPU
box), so this module ships a Treebank-style tokenizer and a lexicon + suffix-rule tagger that
produce the same tag *classes* the selection depends on.  The embedding used for the
distances is pluggable: the scorer's word table or the on-GPU sentence encoder.
"""
from __future__ import annotations

import re
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

# ----------------------------------------------------------------------------- tokenizer
_CONTRACTIONS = [
    (re.compile(r"(?i)\b(can)(not)\b"), r"\1 \2"),
    (re.compile(r"(?i)(\w)(n't)\b"), r"\1 \2"),
    (re.compile(r"(?i)(\w)('s|'re|'ve|'ll|'d|'m)\b"), r"\1 \2"),
]
_PUNCT = re.compile(r"([.,;:!?()\[\]{}\"“”‘’…])")


def word_tokenize(text: str) -> List[str]:
    """Treebank-like tokenisation (the behaviour ``nltk.word_tokenize`` shows on the
    two-sentence prompts this game generates): punctuation split off, contractions split
    (``don't`` → ``do n't``), hyphenated words kept whole, double quotes → ``` `` ``` / ``''``."""
    t = text.replace("\n", " ")
    t = re.sub(r'^"', "`` ", t)
    t = re.sub(r'(\s)"', r"\1`` ", t)
    t = t.replace('"', " '' ")
    t = _PUNCT.sub(r" \1 ", t)
    for pat, rep in _CONTRACTIONS:
        t = pat.sub(rep, t)
    # split a leading/trailing single quote that is not part of a contraction
    toks: List[str] = []
    for tok in t.split():
        if len(tok) > 1 and tok.startswith("'") and tok.lower() not in ("'s", "'re", "'ve", "'ll", "'d", "'m"):
            toks.extend(["'", tok[1:]])
        elif len(tok) > 1 and tok.endswith("'") and not tok.endswith("n'"):
            toks.extend([tok[:-1], "'"])
        else:
            toks.append(tok)
    return toks


def reconstruct_sentence(tokens: Sequence[str]) -> str:
    """Inverse of :func:`word_tokenize` for display.  The reference (``src/utils.py:18-26``)
    also glues hyphenated words to their predecessor; here only punctuation and contraction
    tokens (``n't``, ``'s``, ...) attach without a space."""
    out = ""
    for tok in tokens:
        if (len(tok) == 1 and not tok.isalnum() and tok not in "(`") or tok.startswith("'") or tok.lower() == "n't":
            out += tok
        else:
            out += " " + tok
    return out.strip()


# ----------------------------------------------------------------------------- tagger
_CLOSED: Dict[str, str] = {}


def _add(tag: str, words: str) -> None:
    for w in words.split():
        _CLOSED[w] = tag


_add("DT", "a an the this that these those every each some any no another either neither all both half such")
_add("IN", "of in on at by for with about against between into through during before after above below "
           "from up down over under again further then once beneath beside besides beyond within without "
           "across along amid amidst among amongst around behind toward towards upon onto off past since "
           "until till unto via despite like near throughout underneath inside outside because while "
           "although though if unless whereas whether than as so")
_add("CC", "and or but nor yet plus")
_add("PRP", "i you he she it we they me him her us them myself yourself himself herself itself "
            "ourselves themselves one")
_add("PRP$", "my your his its our their mine yours hers ours theirs")
_add("MD", "can could may might must shall should will would")
_add("TO", "to")
_add("EX", "there")
_add("WDT", "which whatever whichever")
_add("WP", "who whom whose what whoever")
_add("WRB", "when where why how whenever wherever")
_add("VBZ", "is has does seems becomes remains")
_add("VBP", "are am have do")
_add("VBD", "was were had did said went came saw took made knew found gave told became began left felt "
            "brought stood held heard kept ran rose fell grew drew spoke wrote sang flew lay sat shone "
            "struck wove bore tore swept crept slept wept spun sank rang shook woke stole froze broke "
            "chose forgot hid led met paid sent shot spent stuck swam threw understood won wound")
_add("VBN", "been done gone seen taken known given shown grown drawn fallen spoken written woven "
            "frozen broken chosen forgotten hidden stolen")
_add("VBG", "being having doing")
_add("VB", "be")
_add("RB", "not n't very too also just only still even ever never always often soon here there now "
           "then almost quite rather perhaps once twice away back forth together apart ahead aside "
           "yet already else")
_add("RBR", "more less")
_add("RBS", "most least")
_add("JJR", "better worse")
_add("JJS", "best worst")
_add("POS", "'s")
_add("CD", "zero two three four five six seven eight nine ten hundred thousand")

_NN_ENDING_LY = {"family", "lily", "ally", "belly", "bully", "jelly", "folly", "holly", "fly", "rally",
                 "valley", "sally", "gully", "reply", "supply", "assembly", "monopoly", "anomaly"}
_JJ_ENDING_LY = {"lonely", "lovely", "lively", "ghostly", "early", "friendly", "ugly", "holy", "silly",
                 "costly", "deadly", "elderly", "heavenly", "kindly", "likely", "manly", "orderly",
                 "stately", "timely", "unlikely", "worldly", "wobbly", "chilly", "curly", "daily",
                 "only", "otherworldly", "wily"}
_JJ_SUFFIXES = ("ous", "ful", "ive", "able", "ible", "al", "ic", "less", "ish", "ent", "ant", "ary",
                "esque", "ian", "ular", "some", "ine", "ile", "id", "y")
_NN_SUFFIXES = ("tion", "sion", "ness", "ment", "ity", "ship", "hood", "dom", "ism", "ist", "ance",
                "ence", "er", "or", "ure", "age", "scape", "light", "glass", "stone", "wood", "fall")
_JJ_WORDS = set("""
ancient old new young dark bright silent quiet deep vast tiny huge small big great little long short
tall cold warm hot cool soft hard gentle wild strange distant forgotten lost hidden broken golden silver
crimson azure emerald scarlet violet ivory ebony amber pale faint dim radiant luminous shimmering gleaming
glowing eerie haunting sacred mystic mystical arcane celestial astral lunar solar stellar cosmic ethereal
spectral twilight midnight endless infinite eternal fragile fierce brave lone weary restless swift slow
sharp dull bitter sweet sour rich poor empty full hollow heavy light wet dry red blue green black white
grey gray purple orange yellow pink brown dusky misty foggy stormy frozen molten velvet crystal sapphire
ruby obsidian marble iron stone wooden jagged twisted tangled curious ornate barren fertile lush verdant
sunlit moonlit starlit shadowed secret true false strange ancient last first final immortal fallen resonant
whispering duskened snowy sandy dusty rusty misty stony
""".split())


def pos_tag(tokens: Sequence[str]) -> List[Tuple[str, str]]:
    """Lexicon + suffix-rule tagger.  Closed-class words come from a table; open-class words
    are classified by morphology.  Tags use the Penn Treebank names nltk emits."""
    out: List[Tuple[str, str]] = []
    prev = None
    for i, tok in enumerate(tokens):
        low = tok.lower()
        if not any(ch.isalnum() for ch in tok):
            tag = "." if tok in ".!?" else ("," if tok == "," else ":")
        elif tok.replace(".", "", 1).isdigit():
            tag = "CD"
        elif low in _CLOSED:
            tag = _CLOSED[low]
        elif tok[0].isupper() and i > 0 and prev not in (".", "``", ":") and low not in _JJ_WORDS:
            tag = "NNP"
        elif low in _JJ_WORDS:
            tag = "JJ"
        elif low.endswith("ly") and len(low) > 3:
            tag = "NN" if low in _NN_ENDING_LY else ("JJ" if low in _JJ_ENDING_LY else "RB")
        elif low.endswith("est") and len(low) > 5 and low[:-3] + "" in _JJ_WORDS:
            tag = "JJS"
        elif low.endswith("er") and len(low) > 4 and low[:-2] in _JJ_WORDS:
            tag = "JJR"
        elif low.endswith("ing") and len(low) > 4:
            # gerund/participle; after a determiner it is usually a noun/adjective use
            tag = "JJ" if prev in ("DT", "PRP$", "JJ") else "VBG"
        elif low.endswith("ed") and len(low) > 4:
            tag = "JJ" if prev in ("DT", "PRP$", "RB") else "VBD"
        elif low.endswith(_NN_SUFFIXES) and len(low) > 4:
            tag = "NN"
        elif low.endswith(_JJ_SUFFIXES) and len(low) > 4:
            tag = "JJ"
        elif low.endswith("s") and not low.endswith(("ss", "us", "is")) and len(low) > 3:
            tag = "NNS"
        else:
            tag = "NN"
        out.append((tok, tag))
        prev = tag if tag not in ("``",) else tok
    return out


DESCRIPTIVE_TAGS = ("JJ", "RB", "NN", "NNS", "JJR", "JJS", "RBR", "RBS")  # src/utils.py:87

Embedder = Callable[[Sequence[str]], List[Optional[np.ndarray]]]


def semantic_distances(words: Sequence[str], embed: Embedder) -> List[float]:
    """‖v_w − mean(v)‖₂ for each word; 0 for OOV (``src/utils.py:74-79``)."""
    vecs = embed(words)
    known = [v for v in vecs if v is not None]
    if not known:
        return [0.0] * len(words)
    mean = np.mean(np.stack(known), axis=0)
    return [float(np.linalg.norm(v - mean)) if v is not None else 0.0 for v in vecs]


def select_descriptive_words(embed: Embedder, sentence: str, num_words: int = 2,
                             distinct: bool = True) -> Tuple[List[str], List[int]]:
    """Returns ``(tokens, sorted mask indices)``.

    ``distinct=False`` reproduces the reference's ``words.index`` first-occurrence lookup,
    which yields duplicate indices for a repeated word (Appendix C.4).  The default picks
    the highest-scoring *distinct* positions instead.  The TF-IDF factor of the reference is
    identically 1.0 on a single document (Appendix C.5) and is omitted."""
    words = word_tokenize(sentence)
    tagged = pos_tag(words)
    cand = [(i, w) for i, (w, t) in enumerate(tagged) if w.isalpha() and t in DESCRIPTIVE_TAGS]
    if not cand:
        cand = [(i, w) for i, w in enumerate(words) if w.isalpha()]
    if not cand:
        return words, []
    dist = semantic_distances([w for _, w in cand], embed)
    order = np.argsort(np.asarray(dist), kind="stable")
    if distinct:
        picked: List[int] = []
        seen = set()
        for j in order[::-1]:
            idx, w = cand[int(j)]
            if w.lower() in seen:
                continue
            seen.add(w.lower())
            picked.append(idx)
            if len(picked) == num_words:
                break
        return words, sorted(picked)
    top = order[-num_words:]
    return words, sorted(words.index(cand[int(j)][1]) for j in top)


def construct_prompt_dict(embed: Embedder, prompt: str, num_masked: int,
                          distinct: bool = True) -> Dict[str, List]:
    """Canonical round secret ``{'tokens','masks'}`` (``src/utils.py:106-111``)."""
    words, masks = select_descriptive_words(embed, prompt, num_masked, distinct=distinct)
    return {"tokens": words, "masks": masks}


def format_seconds_to_time(seconds: int) -> str:
    """``MM:SS`` (``src/utils.py:28-30``); negative TTLs (missing key) clamp to 00:00."""
    seconds = max(0, int(seconds))
    m, s = divmod(seconds, 60)
    return f"{m:02d}:{s:02d}"
