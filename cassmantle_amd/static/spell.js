// Affix-rule spell checker with suggestions for the guess box (hunspell .aff/.dic subset).
//
// Parity target: the reference client checks every guess with Typo.js over the en_US hunspell
// dictionary (static/script.js:1-10 load, :413-441 hasTypo; typo.js check / suggest).  This is
// our own engine over the grammar tools/build_affix_dict.py writes to /data/words.{aff,dic}:
// PFX/SFX blocks (strip, add, condition, cross-product flag) and stem/FLAGS entries.  It is the
// browser twin of cassmantle_amd/game/spell.py -- same algorithm, same answers (tests/test_spell.py
// runs both under node and compares).
"use strict";

const QWERTY_ROWS = ["qwertyuiop", "asdfghjkl", "zxcvbnm"];
const NEIGHBOURS = (() => {
  const nb = {};
  QWERTY_ROWS.forEach((row, r) => {
    for (let i = 0; i < row.length; i++) {
      let s = "";
      for (const j of [i - 1, i + 1]) if (j >= 0 && j < row.length) s += row[j];
      for (const rr of [r - 1, r + 1]) {
        if (rr < 0 || rr >= QWERTY_ROWS.length) continue;
        for (const j of [i - 1, i, i + 1]) if (j >= 0 && j < QWERTY_ROWS[rr].length) s += QWERTY_ROWS[rr][j];
      }
      nb[row[i]] = s;
    }
  });
  return nb;
})();

class AffixRule {
  constructor(kind, flag, cross, strip, add, cond) {
    this.kind = kind;
    this.flag = flag;
    this.cross = cross;
    this.strip = strip === "0" ? "" : strip;
    this.add = add === "0" ? "" : add.split("/")[0];
    this.cond = new RegExp(kind === "SFX" ? "(" + cond + ")$" : "^(" + cond + ")");
  }

  // the stem this rule would have derived `word` from, or null
  undo(word) {
    let stem;
    if (this.kind === "SFX") {
      if (!word.endsWith(this.add) || word.length <= this.add.length) return null;
      stem = word.slice(0, word.length - this.add.length) + this.strip;
    } else {
      if (!word.startsWith(this.add) || word.length <= this.add.length) return null;
      stem = this.strip + word.slice(this.add.length);
    }
    return this.cond.test(stem) ? stem : null;
  }
}

class AffixSpeller {
  constructor(affText, dicText) {
    this.rules = [];
    this.tryChars = "abcdefghijklmnopqrstuvwxyz";
    const lines = affText.split(/\r?\n/);
    for (let i = 0; i < lines.length;) {
      const p = lines[i].trim().split(/\s+/);
      if (p.length >= 2 && p[0] === "TRY") this.tryChars = p[1];
      if (p.length === 4 && (p[0] === "PFX" || p[0] === "SFX") && (p[2] === "Y" || p[2] === "N")) {
        const n = parseInt(p[3], 10);
        for (let j = 1; j <= n; j++) {
          const q = lines[i + j].trim().split(/\s+/);
          this.rules.push(new AffixRule(p[0], p[1], p[2] === "Y", q[2], q[3], q.length > 4 ? q[4] : "."));
        }
        i += n + 1;
        continue;
      }
      i += 1;
    }
    this.flags = new Map();
    const dl = dicText.split(/\r?\n/);
    const start = dl.length && /^\d+$/.test(dl[0].trim()) ? 1 : 0;
    for (let i = start; i < dl.length; i++) {
      const ln = dl[i].trim();
      if (!ln) continue;
      const k = ln.indexOf("/");
      const stem = k < 0 ? ln : ln.slice(0, k), fl = k < 0 ? "" : ln.slice(k + 1);
      this.flags.set(stem, (this.flags.get(stem) || "") + fl);
    }
    this.sfx = this.rules.filter((r) => r.kind === "SFX");
    this.pfx = this.rules.filter((r) => r.kind === "PFX");
  }

  has(stem, flag) {
    const fl = this.flags.get(stem);
    return fl !== undefined && fl.includes(flag);
  }

  check(word) {
    const w = word.trim().toLowerCase();
    if (!w) return false;
    if (this.flags.has(w)) return true;
    for (const r of this.sfx) {
      const stem = r.undo(w);
      if (stem === null) continue;
      if (this.has(stem, r.flag)) return true;
      if (r.cross) {                      // prefix + suffix on one stem
        for (const p of this.pfx) {
          if (!p.cross) continue;
          const s2 = p.undo(stem);
          if (s2 !== null && this.has(s2, p.flag) && this.has(s2, r.flag)) return true;
        }
      }
    }
    for (const p of this.pfx) {
      const stem = p.undo(w);
      if (stem !== null && this.has(stem, p.flag)) return true;
    }
    return false;
  }

  // [candidate, cost]: transposition 0.5, insertion / deletion 0.8, substitution 0.6 for a
  // QWERTY neighbour and 1.0 otherwise
  edits1(w) {
    const out = [];
    const n = w.length;
    for (let i = 0; i < n; i++) out.push([w.slice(0, i) + w.slice(i + 1), 0.8]);
    for (let i = 0; i < n - 1; i++) out.push([w.slice(0, i) + w[i + 1] + w[i] + w.slice(i + 2), 0.5]);
    for (let i = 0; i < n; i++) {
      const near = NEIGHBOURS[w[i]] || "";
      for (const c of this.tryChars) if (c !== w[i]) out.push([w.slice(0, i) + c + w.slice(i + 1), near.includes(c) ? 0.6 : 1.0]);
    }
    for (let i = 0; i <= n; i++) for (const c of this.tryChars) out.push([w.slice(0, i) + c + w.slice(i), 0.8]);
    return out;
  }

  // corrections ranked by total edit cost (distance 2 only when distance 1 finds nothing and the
  // word is short), then same first letter, then alphabetically
  suggest(word, limit = 5) {
    const w = word.trim().toLowerCase();
    if (!w || this.check(w)) return [];
    const e1 = this.edits1(w);
    const found = new Map();
    for (const [c, cost] of e1) if (c && this.check(c) && cost < (found.has(c) ? found.get(c) : 9.0)) found.set(c, cost);
    if (found.size === 0 && w.length <= 8) {
      const best1 = new Map();
      for (const [c, cost] of e1) if (c && cost < (best1.has(c) ? best1.get(c) : 9.0)) best1.set(c, cost);
      for (const [c, cost] of best1) {
        for (const [c2, cost2] of this.edits1(c)) {
          if (c2 && c2 !== w && cost + cost2 < (found.has(c2) ? found.get(c2) : 9.0) && this.check(c2)) found.set(c2, cost + cost2);
        }
      }
    }
    const ranked = [...found.keys()].sort((a, b) => {
      if (found.get(a) !== found.get(b)) return found.get(a) - found.get(b);
      const fa = a[0] !== w[0] ? 1 : 0, fb = b[0] !== w[0] ? 1 : 0;
      if (fa !== fb) return fa - fb;
      return a < b ? -1 : a > b ? 1 : 0;
    });
    return ranked.slice(0, limit);
  }
}

if (typeof module !== "undefined" && module.exports) module.exports = { AffixSpeller };
