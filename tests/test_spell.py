"""Spell-check parity (reference: Typo.js check / suggest over a hunspell .aff/.dic,
static/script.js:1-10 and 413-441): our affix dictionary reproduces the shipped word list
exactly, check() handles affixed forms, suggest() ranks likely corrections first, the browser
engine (static/spell.js, run under node) gives the same answers as the Python twin, and the
/spell route serves them."""
import json
import os
import shutil
import subprocess

import pytest

from cassmantle_amd.game.spell import AffixSpeller, default_speller

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "cassmantle_amd", "data")
PROBE = ["lantern", "lanterns", "glowing", "unkind", "rebuild", "happily", "happiest", "tower", "towers",
         "crystal", "shadows", "ember", "ancient", "xylophones", "lantren", "lanter", "ambr", "glowng", "shadwo",
         "cystal", "emebr", "riverr", "towre", "qzq", "unhappily", "recrystal", "Lantern", "a", "zz"]


@pytest.fixture(scope="module")
def sp():
    return default_speller()


def test_affix_dictionary_expands_to_the_word_list(sp):
    words = {w.strip() for w in open(os.path.join(DATA, "words.txt")) if w.strip()}
    assert sp.expand() == words
    assert len(sp.flags) < 0.6 * len(words)          # the affix grammar actually compresses


def test_check_affixed_forms(sp):
    for w in ["lantern", "lanterns", "glowing", "unkind", "rebuild", "happily", "Tower", "towers"]:
        assert sp.check(w), w
    for w in ["lantren", "glowng", "qzq", "", "towerz"]:
        assert not sp.check(w), w


def test_suggest_ranks_likely_corrections_first(sp):
    assert sp.suggest("lantren")[0] == "lantern"          # transposition
    assert sp.suggest("lanter")[0] == "lantern"           # missing letter
    assert sp.suggest("glowng")[0] == "glowing"
    assert sp.suggest("shadwo")[0] == "shadow"
    assert sp.suggest("cystal")[0] == "crystal"
    assert sp.suggest("lantern") == []                    # correct words get no suggestions
    assert all(sp.check(w) for w in sp.suggest("ambr"))


def test_grammar_parser_handles_cross_products():
    aff = "SET UTF-8\nTRY abc\nPFX U Y 1\nPFX U 0 un .\nSFX S Y 1\nSFX S 0 s .\n"
    sp = AffixSpeller(aff, "2\nkind/US\ntie\n")
    assert sp.check("unkinds") and sp.check("unkind") and sp.check("kinds") and not sp.check("unties")
    assert sp.expand() == {"kind", "unkind", "kinds", "unkinds", "tie"}


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_browser_engine_matches_python(sp):
    js = f"""
const fs = require("fs");
const {{ AffixSpeller }} = require({json.dumps(os.path.join(ROOT, "cassmantle_amd", "static", "spell.js"))});
const sp = new AffixSpeller(fs.readFileSync({json.dumps(os.path.join(DATA, "words.aff"))}, "utf8"),
                            fs.readFileSync({json.dumps(os.path.join(DATA, "words.dic"))}, "utf8"));
const words = {json.dumps(PROBE)};
console.log(JSON.stringify(words.map((w) => [sp.check(w), sp.suggest(w, 5)])));
"""
    out = subprocess.run(["node", "-e", js], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = json.loads(out.stdout)
    exp = [[sp.check(w), sp.suggest(w, 5)] for w in PROBE]
    assert got == exp


def test_spell_route():
    from tests.test_api import make_client
    client, _ = make_client()
    with client:
        r = client.get("/spell", params={"word": "lantren"}).json()
        assert r["ok"] is False and r["suggestions"][0] == "lantern"
        assert client.get("/spell", params={"word": "lanterns"}).json() == {"word": "lanterns", "ok": True, "suggestions": []}
        assert client.get("/spell", params={"word": "a b"}).json()["ok"] is False
        assert client.get("/static/spell.js").status_code == 200
        assert client.get("/data/words.dic").status_code == 200
