"""Affix-rule spell checker with suggestions (hunspell .aff/.dic subset).

Parity target: the reference client spell-checks every guess with Typo.js over the en_US
hunspell dictionary (``/root/reference/static/script.js:1-10`` load, ``:413-441`` ``hasTypo``;
Typo.js ``check`` / ``suggest``).  This module is the server-side twin of ``static/spell.js``
(same grammar, same algorithm, same answers -- tests/test_spell.py runs both): it reads the
PFX/SFX rule blocks (strip, add, condition; cross-product flag) and ``stem/FLAGS`` entries that
``tools/build_affix_dict.py`` writes for ``data/words.{aff,dic}``, checks a word by undoing at
most one suffix and one prefix, and suggests corrections from edit-distance-1 (then 2) candidates.
"""
from __future__ import annotations

import os
import re
from typing import Dict, List, Optional, Sequence, Set, Tuple

_DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


class AffixRule:
    __slots__ = ("kind", "flag", "cross", "strip", "add", "cond")

    def __init__(self, kind: str, flag: str, cross: bool, strip: str, add: str, cond: str):
        self.kind, self.flag, self.cross = kind, flag, cross
        self.strip = "" if strip == "0" else strip
        self.add = "" if add == "0" else add.split("/")[0]
        pat = "(" + cond + ")$" if kind == "SFX" else "^(" + cond + ")"
        self.cond = re.compile(pat)

    def undo(self, word: str) -> Optional[str]:
        """the stem this rule would have derived ``word`` from, or None"""
        if self.kind == "SFX":
            if not word.endswith(self.add) or len(word) <= len(self.add):
                return None
            stem = word[: len(word) - len(self.add)] + self.strip
        else:
            if not word.startswith(self.add) or len(word) <= len(self.add):
                return None
            stem = self.strip + word[len(self.add):]
        return stem if self.cond.search(stem) else None


class AffixSpeller:
    def __init__(self, aff_text: str, dic_text: str):
        self.rules: List[AffixRule] = []
        self.try_chars = "abcdefghijklmnopqrstuvwxyz"
        lines = aff_text.splitlines()
        i = 0
        while i < len(lines):
            parts = lines[i].split()
            if len(parts) >= 2 and parts[0] == "TRY":
                self.try_chars = parts[1]
            if len(parts) == 4 and parts[0] in ("PFX", "SFX") and parts[2] in ("Y", "N"):
                kind, flag, cross, n = parts[0], parts[1], parts[2] == "Y", int(parts[3])
                for j in range(1, n + 1):
                    p = lines[i + j].split()
                    self.rules.append(AffixRule(kind, flag, cross, p[2], p[3], p[4] if len(p) > 4 else "."))
                i += n + 1
                continue
            i += 1
        self.flags: Dict[str, str] = {}
        dl = dic_text.splitlines()
        for ln in dl[1:] if dl and dl[0].strip().isdigit() else dl:
            ln = ln.strip()
            if not ln:
                continue
            stem, _, fl = ln.partition("/")
            self.flags[stem] = self.flags.get(stem, "") + fl
        self.sfx = [r for r in self.rules if r.kind == "SFX"]
        self.pfx = [r for r in self.rules if r.kind == "PFX"]
        # rules indexed by their affix string: a rule whose affix is not at the word's end
        # (start) cannot undo it, so check() only tries the few that can (same answers as
        # scanning every rule; ADVICE r2: distance-2 suggestions ran ~200k full scans)
        self._sfx_by_add: Dict[str, List[AffixRule]] = {}
        self._pfx_by_add: Dict[str, List[AffixRule]] = {}
        for r in self.sfx:
            self._sfx_by_add.setdefault(r.add, []).append(r)
        for r in self.pfx:
            self._pfx_by_add.setdefault(r.add, []).append(r)
        self._sfx_lens = sorted({len(a) for a in self._sfx_by_add})
        self._pfx_lens = sorted({len(a) for a in self._pfx_by_add})
        self._check_cache: Dict[str, bool] = {}

    @classmethod
    def load(cls, prefix: Optional[str] = None) -> "AffixSpeller":
        prefix = prefix or os.path.join(_DATA, "words")
        with open(prefix + ".aff") as a, open(prefix + ".dic") as d:
            return cls(a.read(), d.read())

    def _has(self, stem: str, flag: str) -> bool:
        fl = self.flags.get(stem)
        return fl is not None and flag in fl

    def _candidates(self, w: str, by_add, lens, suffix: bool):
        for L in lens:
            if L >= len(w):
                break
            key = w[len(w) - L:] if suffix else w[:L]
            yield from by_add.get(key, ())

    def check(self, word: str) -> bool:
        w = word.strip().lower()
        if not w:
            return False
        hit = self._check_cache.get(w)
        if hit is None:
            hit = self._check(w)
            if len(self._check_cache) > (1 << 20):
                self._check_cache.clear()
            self._check_cache[w] = hit
        return hit

    def _check(self, w: str) -> bool:
        if w in self.flags:
            return True
        for r in self._candidates(w, self._sfx_by_add, self._sfx_lens, True):
            stem = r.undo(w)
            if stem is None:
                continue
            if self._has(stem, r.flag):
                return True
            if r.cross:                        # prefix + suffix on one stem
                for p in self._candidates(stem, self._pfx_by_add, self._pfx_lens, False):
                    if p.cross:
                        s2 = p.undo(stem)
                        if s2 is not None and self._has(s2, p.flag) and self._has(s2, r.flag):
                            return True
        for p in self._candidates(w, self._pfx_by_add, self._pfx_lens, False):
            stem = p.undo(w)
            if stem is not None and self._has(stem, p.flag):
                return True
        return False

    def _edits1(self, w: str) -> List[Tuple[str, float]]:
        """(candidate, cost): transposition 0.5, insertion / deletion 0.8, substitution 0.6 for
        a QWERTY neighbour and 1.0 otherwise (typing-error likelihood order)"""
        out: List[Tuple[str, float]] = []
        n = len(w)
        for i in range(n):                                   # deletions
            out.append((w[:i] + w[i + 1:], 0.8))
        for i in range(n - 1):                               # adjacent transpositions
            out.append((w[:i] + w[i + 1] + w[i] + w[i + 2:], 0.5))
        for i in range(n):                                   # substitutions
            near = _NEIGHBOURS.get(w[i], "")
            for c in self.try_chars:
                if c != w[i]:
                    out.append((w[:i] + c + w[i + 1:], 0.6 if c in near else 1.0))
        for i in range(n + 1):                               # insertions
            for c in self.try_chars:
                out.append((w[:i] + c + w[i:], 0.8))
        return out

    def suggest(self, word: str, limit: int = 5) -> List[str]:
        """corrections ranked by total edit cost (distance-2 candidates only when distance 1
        finds nothing), then same first letter, then alphabetically"""
        w = word.strip().lower()
        if not w or self.check(w):
            return []
        e1 = self._edits1(w)
        found: Dict[str, float] = {}
        for c, cost in e1:
            if c and self.check(c) and cost < found.get(c, 9.0):
                found[c] = cost
        if not found and len(w) <= 8:
            best1: Dict[str, float] = {}
            for c, cost in e1:
                if c and cost < best1.get(c, 9.0):
                    best1[c] = cost
            for c, cost in best1.items():
                for c2, cost2 in self._edits1(c):
                    if c2 and c2 != w and cost + cost2 < found.get(c2, 9.0) and self.check(c2):
                        found[c2] = cost + cost2
        ranked = sorted(found, key=lambda c: (found[c], c[0] != w[0], c))
        return ranked[:limit]

    def expand(self) -> Set[str]:
        """every word the dictionary accepts through single affixes (cross products included)"""
        out: Set[str] = set()
        for stem, fl in self.flags.items():
            out.add(stem)
            for r in self.rules:
                if r.flag not in fl:
                    continue
                w = self._apply(r, stem)
                if w is None:
                    continue
                out.add(w)
                if r.kind == "SFX" and r.cross:
                    for p in self.pfx:
                        if p.cross and p.flag in fl:
                            w2 = self._apply(p, w)
                            if w2 is not None:
                                out.add(w2)
        return out

    @staticmethod
    def _apply(r: AffixRule, stem: str) -> Optional[str]:
        if not r.cond.search(stem):
            return None
        if r.kind == "SFX":
            if r.strip and not stem.endswith(r.strip):
                return None
            return stem[: len(stem) - len(r.strip)] + r.add
        if r.strip and not stem.startswith(r.strip):
            return None
        return r.add + stem[len(r.strip):]


_ROWS = ("qwertyuiop", "asdfghjkl", "zxcvbnm")
_NEIGHBOURS: Dict[str, str] = {}
for _r, _row in enumerate(_ROWS):
    for _i, _ch in enumerate(_row):
        _nb = [_row[j] for j in (_i - 1, _i + 1) if 0 <= j < len(_row)]
        for _rr in (_r - 1, _r + 1):
            if 0 <= _rr < len(_ROWS):
                _nb += [_ROWS[_rr][j] for j in (_i - 1, _i, _i + 1) if 0 <= j < len(_ROWS[_rr])]
        _NEIGHBOURS[_ch] = "".join(_nb)

_DEFAULT: Optional[AffixSpeller] = None


def default_speller() -> AffixSpeller:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = AffixSpeller.load()
    return _DEFAULT


def spell_report(word: str, limit: int = 5) -> Dict[str, object]:
    sp = default_speller()
    ok = sp.check(word)
    return {"word": word, "ok": ok, "suggestions": [] if ok else sp.suggest(word, limit)}
