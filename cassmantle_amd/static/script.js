// CassMantle browser client.
// Talks to the API contract of SURVEY Appendix A: /client/status, /init, /clock (WS),
// /fetch/contents, /compute_score.  Behaviour follows the reference client
// (static/script.js in SnowCheetos/CassMantle): spell-checked guesses, per-mask score
// placeholders ("try again" at <= 0.1), solved words shown in green, win message, blinking
// clock under one minute, refetch on the round-reset flag.
"use strict";

const EPISODES = 20;
const params = new URLSearchParams(window.location.search);
const ROOM = params.get("room");
const q = (path) => (ROOM ? `${path}${path.includes("?") ? "&" : "?"}room=${encodeURIComponent(ROOM)}` : path);

let dictionary = null;           // AffixSpeller (static/spell.js) over /data/words.{aff,dic}
let clockSocket = null;

async function loadDictionary() {
  try {
    const [aff, dic] = await Promise.all([fetch("/data/words.aff").then((r) => r.text()),
                                          fetch("/data/words.dic").then((r) => r.text())]);
    dictionary = new AffixSpeller(aff, dic);
  } catch (e) {
    dictionary = null;  // spell-check disabled if the dictionary is unavailable
  }
}

function $(id) { return document.getElementById(id); }

async function getJSON(path, opts) {
  const res = await fetch(q(path), Object.assign({ credentials: "include" }, opts || {}));
  if (res.status === 429) throw new Error("slow down");
  return res.json();
}

async function ensureSession() {
  const st = await getJSON("/client/status");
  if (st.needInitialization) await getJSON("/init");
}

function openClock() {
  const proto = window.location.protocol === "https:" ? "wss" : "ws";
  clockSocket = new WebSocket(`${proto}://${window.location.host}${q("/clock")}`);
  clockSocket.onmessage = (ev) => {
    const msg = JSON.parse(ev.data);
    updateClock(msg.time);
    $("player-count").textContent = msg.conns;
    if (msg.reset) {
      $("status").textContent = "";
      fetchContents();
    }
  };
  clockSocket.onclose = () => setTimeout(openClock, 2000);
}

function updateClock(t) {
  const el = $("clock");
  el.textContent = t;
  const [m] = t.split(":").map(Number);
  el.classList.toggle("urgent", m < 1);
}

function renderStory(story) {
  if (!story) return;
  $("story-title").textContent = story.title || "CassMantle";
  $("story-episode").textContent = story.episode ? `${story.episode}/${EPISODES}` : "";
}

function scoreLabel(s) {
  const v = parseFloat(s);
  if (!(v > 0)) return "";
  if (v <= 0.1) return "try again";
  return (v * 100).toFixed(2);
}

function renderPrompt(p) {
  const box = $("prompt");
  box.innerHTML = "";
  const masks = new Set(p.masks.filter((m) => m >= 0));
  const correct = new Set(p.correct || []);
  p.tokens.forEach((tok, i) => {
    if (masks.has(i)) {
      const inp = document.createElement("input");
      inp.type = "text";
      inp.className = "guess";
      inp.dataset.index = String(i);
      inp.autocomplete = "off";
      inp.placeholder = scoreLabel(p.scores ? p.scores[String(i)] : "");
      inp.addEventListener("keydown", (e) => { if (e.key === "Enter") submitGuesses(); });
      box.appendChild(inp);
    } else {
      const span = document.createElement("span");
      span.textContent = tok;
      if (correct.has(i)) span.className = "solved";
      box.appendChild(span);
    }
    box.appendChild(document.createTextNode(" "));
  });
  const won = p.masks.length === 0 && p.tokens.length > 0;
  $("submit").disabled = won;
  if (won) {
    const n = p.attempts;
    $("status").textContent = `Congratulations, you got it in ${n} attempt${n === 1 ? "" : "s"}!`;
  }
}

async function fetchContents() {
  try {
    const c = await getJSON("/fetch/contents");
    $("round-image").src = `data:image/jpeg;base64,${c.image}`;
    renderStory(c.story);
    renderPrompt(c.prompt);
  } catch (e) {
    $("status").textContent = e.message;
  }
}

function flashRed(el) {
  el.classList.add("invalid");
  setTimeout(() => el.classList.remove("invalid"), 600);
}

function validGuess(v) {
  if (!v || /\s/.test(v) || /[^A-Za-z'-]/.test(v)) return false;
  if (dictionary && !dictionary.check(v)) return false;
  return true;
}

// typo hint under the guess boxes: "did you mean ...?" (click a suggestion to take it)
function showSuggestions(inp) {
  const box = $("suggest");
  if (!box) return;
  box.textContent = "";
  const v = inp.value.trim();
  if (!dictionary || !v || /[^A-Za-z]/.test(v)) return;
  const sug = dictionary.suggest(v, 3);
  if (!sug.length) return;
  box.append(`"${v}" is not in the dictionary. Did you mean `);
  sug.forEach((w, i) => {
    const a = document.createElement("a");
    a.href = "#";
    a.textContent = w;
    a.addEventListener("click", (e) => { e.preventDefault(); inp.value = w; box.textContent = ""; });
    box.append(a, i + 1 < sug.length ? ", " : "?");
  });
}

async function submitGuesses() {
  const inputs = Array.from(document.querySelectorAll("input.guess"));
  const payload = {};
  let ok = true;
  for (const inp of inputs) {
    const v = inp.value.trim();
    if (!validGuess(v)) { flashRed(inp); showSuggestions(inp); ok = false; continue; }
    payload[inp.dataset.index] = v;
  }
  if (!ok || Object.keys(payload).length === 0) return;
  try {
    await getJSON("/compute_score", {
      method: "POST",
      headers: { "Content-Type": "application/json" },
      body: JSON.stringify({ inputs: payload }),
    });
    await fetchContents();
  } catch (e) {
    $("status").textContent = e.message;
  }
}

async function startApp() {
  await Promise.all([loadDictionary(), ensureSession()]);
  openClock();
  await fetchContents();
  $("splash").hidden = true;
}

function setupChrome() {
  $("submit").addEventListener("click", submitGuesses);
  $("privacy-link").addEventListener("click", (e) => { e.preventDefault(); $("privacy-modal").hidden = false; });
  $("privacy-close").addEventListener("click", () => { $("privacy-modal").hidden = true; });
  if (localStorage.getItem("cookiesAccepted")) {
    startApp();
  } else {
    $("cookie-banner").hidden = false;
    $("cookie-accept").addEventListener("click", () => {
      localStorage.setItem("cookiesAccepted", "1");
      $("cookie-banner").hidden = true;
      startApp();
    });
  }
}

document.addEventListener("DOMContentLoaded", setupChrome);
