"""Compress the shipped word list (cassmantle_amd/data/words.txt) into a hunspell-format affix
dictionary (data/words.aff + data/words.dic) for the browser spell checker (static/spell.js) and
its Python twin (cassmantle_amd/game/spell.py).

Parity target: the reference checks guesses with Typo.js against the en_US hunspell .aff/.dic
(/root/reference/static/script.js:1-10, 413-441; typo.js check/suggest).  This tool writes OUR
OWN small affix grammar (plural, past, gerund, comparative, superlative, -ly, -ness, un-, re-)
and greedily moves every word that one rule derives from a kept stem into a flag on that stem.
Within a flag the rule conditions are mutually exclusive and prefixes do not cross with
suffixes, so every (stem, flag) pair expands to exactly one word: the expansion of the
dictionary is EXACTLY the word list (checked here and in tests/test_spell.py).

    python tools/build_affix_dict.py [words.txt] [out_prefix]
"""
from __future__ import annotations

import os
import re
import sys

# flag -> (kind, [(strip, add, condition regex on the STEM)])
RULES = {
    "S": ("SFX", [("y", "ies", "[^aeiou]y"), ("0", "s", "[aeiou]y"), ("0", "es", "[sxzh]"), ("0", "s", "[^sxzhy]")]),
    "D": ("SFX", [("0", "d", "e"), ("y", "ied", "[^aeiou]y"), ("0", "ed", "[aeiou]y"), ("0", "ed", "[^ey]")]),
    "G": ("SFX", [("e", "ing", "e"), ("0", "ing", "[^e]")]),
    "R": ("SFX", [("0", "r", "e"), ("y", "ier", "[^aeiou]y"), ("0", "er", "[aeiou]y"), ("0", "er", "[^ey]")]),
    "T": ("SFX", [("0", "st", "e"), ("y", "iest", "[^aeiou]y"), ("0", "est", "[aeiou]y"), ("0", "est", "[^ey]")]),
    "Y": ("SFX", [("0", "ly", "[^y]"), ("y", "ily", "y")]),
    "N": ("SFX", [("0", "ness", "[^y]"), ("y", "iness", "y")]),
    "U": ("PFX", [("0", "un", ".")]),
    "A": ("PFX", [("0", "re", ".")]),
}
ORDER = "SDGRTYNUA"


def apply_rule(kind, strip, add, cond, stem):
    """the derived word, or None when the rule does not apply to the stem"""
    s = "" if strip == "0" else strip
    if kind == "SFX":
        if not re.search("(" + cond + ")$", stem):
            return None
        if s and not stem.endswith(s):
            return None
        return stem[: len(stem) - len(s)] + add
    if not re.match("^(" + cond + ")", stem):
        return None
    if s and not stem.startswith(s):
        return None
    return add + stem[len(s):]


def derive(stem, flag):
    kind, rules = RULES[flag]
    for strip, add, cond in rules:
        w = apply_rule(kind, strip, add, cond, stem)
        if w is not None:
            return w           # conditions are mutually exclusive: at most one rule applies
    return None


def compress(words):
    wordset = set(words)
    flags = {}                 # kept stem -> set of flags
    for w in sorted(wordset, key=lambda x: (len(x), x)):
        placed = False
        for flag in ORDER:
            kind, rules = RULES[flag]
            for strip, add, cond in rules:
                s = "" if strip == "0" else strip
                if kind == "SFX":
                    if not w.endswith(add) or len(w) <= len(add):
                        continue
                    stem = w[: len(w) - len(add)] + s
                else:
                    if not w.startswith(add) or len(w) <= len(add):
                        continue
                    stem = s + w[len(add):]
                if stem in flags and flag not in flags[stem] and derive(stem, flag) == w:
                    flags[stem].add(flag)
                    placed = True
                    break
            if placed:
                break
        if not placed:
            flags[w] = set()
    return flags


def expand(flags):
    out = set()
    for stem, fl in flags.items():
        out.add(stem)
        for f in fl:
            out.add(derive(stem, f))
    return out


def write(flags, prefix):
    with open(prefix + ".aff", "w") as f:
        f.write("# cassmantle_amd affix grammar (tools/build_affix_dict.py); hunspell syntax\n")
        f.write("SET UTF-8\nTRY esiarntolcdugmphbyfvkwzxjq\n\n")
        for flag in ORDER:
            kind, rules = RULES[flag]
            f.write(f"{kind} {flag} N {len(rules)}\n")
            for strip, add, cond in rules:
                f.write(f"{kind} {flag} {strip} {add} {cond}\n")
            f.write("\n")
    with open(prefix + ".dic", "w") as f:
        f.write(f"{len(flags)}\n")
        for stem in sorted(flags):
            fl = "".join(sorted(flags[stem], key=ORDER.index))
            f.write(f"{stem}/{fl}\n" if fl else f"{stem}\n")


def main():
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cassmantle_amd", "data")
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "words.txt")
    prefix = sys.argv[2] if len(sys.argv) > 2 else os.path.join(here, "words")
    words = [w.strip() for w in open(src) if w.strip()]
    flags = compress(words)
    assert expand(flags) == set(words), "affix expansion must reproduce the word list exactly"
    write(flags, prefix)
    print(f"{len(words)} words -> {len(flags)} stems ({100 * len(flags) / len(words):.1f}%)")


if __name__ == "__main__":
    main()
