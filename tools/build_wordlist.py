"""Expand a hunspell dictionary (.dic + .aff) into a flat word list.

The reference's browser client spell-checks guesses with the vendored Typo.js against
``data/en_US.dic``/``en_US.aff`` (``static/script.js:1-10``, ``static/typo.js``).  This
framework instead ships the *expanded* word list once (``cassmantle_amd/data/words.txt``):
the client checks membership in a ``Set`` and the server uses the same list as the scorer's
vocabulary.  This tool applies PFX/SFX rules (including cross-product prefix+suffix) and
keeps lower-case alphabetic words.

    python tools/build_wordlist.py /path/en_US.aff /path/en_US.dic cassmantle_amd/data/words.txt
"""
from __future__ import annotations

import re
import sys
from typing import Dict, List, Tuple

Rule = Tuple[str, str, "re.Pattern"]  # (strip, add, condition)


def parse_aff(path: str):
    pfx: Dict[str, Tuple[bool, List[Rule]]] = {}
    sfx: Dict[str, Tuple[bool, List[Rule]]] = {}
    with open(path, encoding="utf-8", errors="replace") as f:
        lines = [ln.rstrip("\n") for ln in f]
    i = 0
    while i < len(lines):
        parts = lines[i].split()
        if len(parts) == 4 and parts[0] in ("PFX", "SFX") and parts[2] in ("Y", "N"):
            kind, flag, cross, n = parts[0], parts[1], parts[2] == "Y", int(parts[3])
            rules: List[Rule] = []
            for j in range(1, n + 1):
                p = lines[i + j].split()
                strip = "" if p[2] == "0" else p[2]
                add = "" if p[3] == "0" else p[3].split("/")[0]
                cond = p[4] if len(p) > 4 else "."
                pat = re.compile(("^" + cond) if kind == "PFX" else (cond + "$"))
                rules.append((strip, add, pat))
            (pfx if kind == "PFX" else sfx)[flag] = (cross, rules)
            i += n + 1
            continue
        i += 1
    return pfx, sfx


def expand(word: str, flags: str, pfx, sfx) -> List[str]:
    out = [word]
    suffixed: List[Tuple[str, bool]] = []
    for fl in flags:
        if fl in sfx:
            cross, rules = sfx[fl]
            for strip, add, pat in rules:
                if pat.search(word) and (not strip or word.endswith(strip)):
                    w = (word[: len(word) - len(strip)] if strip else word) + add
                    out.append(w)
                    suffixed.append((w, cross))
    for fl in flags:
        if fl in pfx:
            cross, rules = pfx[fl]
            for strip, add, pat in rules:
                if pat.search(word) and (not strip or word.startswith(strip)):
                    out.append(add + (word[len(strip):] if strip else word))
                if cross:
                    for w, c in suffixed:
                        if c and pat.search(w):
                            out.append(add + (w[len(strip):] if strip else w))
    return out


def main(aff: str, dic: str, dst: str) -> int:
    pfx, sfx = parse_aff(aff)
    words = set()
    with open(dic, encoding="utf-8", errors="replace") as f:
        next(f)
        for ln in f:
            ln = ln.strip()
            if not ln:
                continue
            w, _, fl = ln.partition("/")
            for x in expand(w, fl, pfx, sfx):
                if x.isalpha() and x.isascii():
                    words.add(x.lower())
    with open(dst, "w", encoding="utf-8") as f:
        for w in sorted(words):
            f.write(w + "\n")
    print(f"wrote {len(words)} words to {dst}")
    return 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:4]))
