"""In-process state store with the Redis subset the reference uses.

Reference: every piece of shared state lives in a Redis server reached over TCP
(``src/backend.py:70-71``) — hashes ``prompt``/``image``/``story``/``<session>``, the set
``sessions``, TTL keys ``countdown``/``reset`` and three ``SET NX PX`` locks (SURVEY
Appendix B).  Here the front-end process owns the game state, so the store is a plain
in-memory structure driven by an injectable :class:`~cassmantle_amd.game.clock.Clock`.
The method names and return conventions follow Redis (``TTL`` returns -2 for a missing key,
-1 for no expiry) so the game logic reads like the reference's, but values are ``str`` (the
reference decodes bytes everywhere) except for raw ``bytes`` payloads (JPEGs).

Thread safety: the event loop is the main user, but worker threads (``asyncio.to_thread`` blur
/ JPEG work, generation callbacks) touch it too, so every operation runs under one re-entrant
mutex (expiry bookkeeping in ``_alive`` mutates the dicts even on reads).  Multi-step
read-modify-write sequences that the reference leaves racy (``set_client_scores``,
``src/server.py:79-82``) are made atomic across coroutines with :meth:`StateStore.critical`
(SURVEY §5.2).
"""
from __future__ import annotations

import asyncio
import base64
import contextlib
import functools
import json
import threading
import uuid
from typing import Any, Dict, Iterable, Optional, Set, Union

from .clock import Clock

Value = Union[str, bytes]


class LockError(Exception):
    """Raised when a lock cannot be acquired within ``blocking_timeout`` (aioredis parity)."""


def _enc(v: Any) -> Value:
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    if isinstance(v, bool):
        return str(int(v))
    return str(v)


def _synchronized(fn):
    @functools.wraps(fn)
    def wrapper(self, *a, **kw):
        with self._mu:
            return fn(self, *a, **kw)
    return wrapper


class StateStore:
    def __init__(self, clock: Optional[Clock] = None) -> None:
        self._mu = threading.RLock()
        self.clock = clock or Clock()
        self._data: Dict[str, Any] = {}
        self._expiry: Dict[str, float] = {}
        self._locks: Dict[str, tuple] = {}
        self._crit: Dict[str, asyncio.Lock] = {}
        self.ops = 0  # operation counter (metrics)

    # ------------------------------------------------------------------ expiry
    @_synchronized
    def _alive(self, key: str) -> bool:
        exp = self._expiry.get(key)
        if exp is not None and self.clock.now() >= exp:
            self._data.pop(key, None)
            self._expiry.pop(key, None)
            return False
        return key in self._data

    @_synchronized
    def _get(self, key: str, typ: type) -> Any:
        self.ops += 1
        if not self._alive(key):
            return None
        v = self._data[key]
        if not isinstance(v, typ):
            raise TypeError(f"WRONGTYPE key {key}")
        return v

    # ------------------------------------------------------------------ keys
    @_synchronized
    def exists(self, *keys: str) -> int:
        self.ops += 1
        return sum(1 for k in keys if k is not None and self._alive(k))

    @_synchronized
    def delete(self, *keys: str) -> int:
        n = 0
        for k in keys:
            if self._alive(k):
                n += 1
            self._data.pop(k, None)
            self._expiry.pop(k, None)
        return n

    @_synchronized
    def expire(self, key: str, seconds: float) -> bool:
        if not self._alive(key):
            return False
        self._expiry[key] = self.clock.now() + float(seconds)
        return True

    @_synchronized
    def ttl(self, key: str) -> int:
        """Redis TTL: integer seconds remaining (rounded like Redis: ceil of ms/1000 rounded
        to nearest), -2 if missing, -1 if no expiry."""
        self.ops += 1
        if not self._alive(key):
            return -2
        exp = self._expiry.get(key)
        if exp is None:
            return -1
        rem = exp - self.clock.now()
        return int(rem + 0.5)

    @_synchronized
    def pttl(self, key: str) -> float:
        if not self._alive(key):
            return -2
        exp = self._expiry.get(key)
        return -1 if exp is None else (exp - self.clock.now())

    # ------------------------------------------------------------------ strings
    @_synchronized
    def set(self, key: str, value: Any, ex: Optional[float] = None, nx: bool = False) -> bool:
        if nx and self._alive(key):
            return False
        self._data[key] = _enc(value)
        if ex is not None:
            self._expiry[key] = self.clock.now() + float(ex)
        else:
            self._expiry.pop(key, None)
        return True

    @_synchronized
    def setex(self, key: str, seconds: float, value: Any) -> bool:
        return self.set(key, value, ex=seconds)

    @_synchronized
    def get(self, key: str) -> Optional[Value]:
        return self._get(key, (str, bytes))

    # ------------------------------------------------------------------ hashes
    @_synchronized
    def hset(self, key: str, field: Optional[str] = None, value: Any = None,
             mapping: Optional[Dict[str, Any]] = None) -> int:
        h = self._get(key, dict)
        if h is None:
            h = {}
            self._data[key] = h
        n = 0
        items = dict(mapping or {})
        if field is not None:
            items[field] = value
        for f, v in items.items():
            f = str(f)
            if f not in h:
                n += 1
            h[f] = _enc(v)
        return n

    @_synchronized
    def hget(self, key: str, field: str) -> Optional[Value]:
        h = self._get(key, dict)
        return None if h is None else h.get(str(field))

    @_synchronized
    def hgetall(self, key: str) -> Dict[str, Value]:
        h = self._get(key, dict)
        return {} if h is None else dict(h)

    @_synchronized
    def hdel(self, key: str, *fields_: str) -> int:
        h = self._get(key, dict)
        if h is None:
            return 0
        n = 0
        for f in fields_:
            if h.pop(str(f), None) is not None:
                n += 1
        if not h:
            self.delete(key)
        return n

    @_synchronized
    def hincrby(self, key: str, field: str, amount: int = 1) -> int:
        h = self._get(key, dict)
        if h is None:
            h = {}
            self._data[key] = h
        cur = int(h.get(field, "0"))
        cur += int(amount)
        h[field] = str(cur)
        return cur

    @_synchronized
    def hexists(self, key: str, field: str) -> bool:
        h = self._get(key, dict)
        return h is not None and str(field) in h

    # ------------------------------------------------------------------ sets
    @_synchronized
    def sadd(self, key: str, *members: str) -> int:
        s = self._get(key, set)
        if s is None:
            s = set()
            self._data[key] = s
        n = 0
        for m in members:
            if m not in s:
                s.add(m)
                n += 1
        return n

    @_synchronized
    def srem(self, key: str, *members: str) -> int:
        s = self._get(key, set)
        if s is None:
            return 0
        n = 0
        for m in members:
            if m in s:
                s.discard(m)
                n += 1
        return n

    @_synchronized
    def smembers(self, key: str) -> Set[str]:
        s = self._get(key, set)
        return set() if s is None else set(s)

    @_synchronized
    def sismember(self, key: str, member: str) -> bool:
        s = self._get(key, set)
        return s is not None and member in s

    @_synchronized
    def scard(self, key: str) -> int:
        s = self._get(key, set)
        return 0 if s is None else len(s)

    # ------------------------------------------------------------------ locks
    @contextlib.asynccontextmanager
    async def lock(self, name: str, timeout: float = 120.0, blocking_timeout: float = 2.0):
        """``SET NX PX`` lock with expiry (aioredis ``Lock`` parity, ``src/backend.py:83``).

        A crashed holder's lock expires after ``timeout`` seconds of store-clock time.
        Raises :class:`LockError` if not acquired within ``blocking_timeout``."""
        token = uuid.uuid4().hex
        deadline = self.clock.now() + blocking_timeout
        while True:
            if self.set(name, token, ex=timeout, nx=True):
                break
            if self.clock.now() >= deadline:
                raise LockError(name)
            await self.clock.sleep(0.05)
        try:
            yield token
        finally:
            if self._alive(name) and self._data.get(name) == token:
                self.delete(name)

    def critical(self, name: str) -> asyncio.Lock:
        """In-process mutex for multi-step read-modify-write sequences."""
        lk = self._crit.get(name)
        if lk is None:
            lk = asyncio.Lock()
            self._crit[name] = lk
        return lk

    # ------------------------------------------------------------------ snapshot
    @_synchronized
    def snapshot(self) -> Dict[str, Any]:
        """JSON-serialisable dump (checkpoint/resume).  TTLs are stored as
        remaining seconds so they survive a restart on a different clock."""
        out: Dict[str, Any] = {}
        now = self.clock.now()
        for k in list(self._data):
            if not self._alive(k):
                continue
            v = self._data[k]
            if isinstance(v, dict):
                enc = {"t": "hash", "v": {f: _wire(x) for f, x in v.items()}}
            elif isinstance(v, set):
                enc = {"t": "set", "v": sorted(v)}
            else:
                enc = {"t": "str", "v": _wire(v)}
            exp = self._expiry.get(k)
            if exp is not None:
                enc["ttl"] = exp - now
            out[k] = enc
        return out

    @_synchronized
    def restore(self, snap: Dict[str, Any]) -> None:
        self._data.clear()
        self._expiry.clear()
        now = self.clock.now()
        for k, enc in snap.items():
            t = enc["t"]
            if t == "hash":
                self._data[k] = {f: _unwire(x) for f, x in enc["v"].items()}
            elif t == "set":
                self._data[k] = set(enc["v"])
            else:
                self._data[k] = _unwire(enc["v"])
            if "ttl" in enc:
                self._expiry[k] = now + float(enc["ttl"])

    def dumps(self) -> str:
        return json.dumps(self.snapshot())

    def loads(self, s: str) -> None:
        self.restore(json.loads(s))


def _wire(v: Value) -> Any:
    if isinstance(v, bytes):
        return {"b64": base64.b64encode(v).decode()}
    return v


def _unwire(v: Any) -> Value:
    if isinstance(v, dict) and "b64" in v:
        return base64.b64decode(v["b64"])
    return v
