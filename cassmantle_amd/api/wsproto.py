"""Minimal RFC 6455 WebSocket server protocol for uvicorn (no third-party websocket library).

The reference serves its ``/clock`` socket through uvicorn with the ``websockets`` package
(``main.py:55-79``, ``requirements.txt:2``).  Neither ``websockets`` nor ``wsproto`` exists on
the serving image, so uvicorn's h11 HTTP protocol hands upgrade requests to this class
(``uvicorn.run(..., ws="cassmantle_amd.api.wsproto:RFC6455Protocol")``).  It implements what the
game needs and browsers send: the opening handshake, masked client frames (text, binary,
continuation), ping/pong, close, and the ASGI ``websocket.*`` message interface.  No
extensions (permessage-deflate is declined by omission, which RFC 6455 allows).
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import logging
import struct
from typing import Any, Dict, List, Optional, Tuple
from urllib.parse import unquote

log = logging.getLogger("cassmantle")
_GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"
MAX_MESSAGE = 1 << 20          # largest frame AND largest reassembled message
MAX_HANDSHAKE = 16 << 10       # request line + headers
MAX_QUEUED = 64                # received messages not yet taken by the application


def accept_key(key: bytes) -> bytes:
    return base64.b64encode(hashlib.sha1(key.strip() + _GUID).digest())


def encode_frame(opcode: int, payload: bytes, fin: bool = True) -> bytes:
    """Server -> client frame (never masked)."""
    b0 = (0x80 if fin else 0) | opcode
    n = len(payload)
    if n < 126:
        head = struct.pack("!BB", b0, n)
    elif n < (1 << 16):
        head = struct.pack("!BBH", b0, 126, n)
    else:
        head = struct.pack("!BBQ", b0, 127, n)
    return head + payload


class FrameParser:
    """Incremental client-frame decoder.  ``feed`` returns complete (opcode, payload) messages
    (continuations reassembled; control frames returned as they arrive).  Raises ``ValueError``
    (-> close 1002) on protocol errors: an unmasked client frame (RFC 6455 §5.1), a frame or a
    reassembled message over ``MAX_MESSAGE``, a fragmented or oversized control frame, or a
    continuation without a start."""

    def __init__(self, require_mask: bool = True) -> None:
        self.require_mask = require_mask     # False only to decode server -> client frames
        self.buf = bytearray()
        self.frag_op: Optional[int] = None
        self.frag: List[bytes] = []
        self.frag_len = 0

    def feed(self, data: bytes) -> List[Tuple[int, bytes]]:
        self.buf += data
        out: List[Tuple[int, bytes]] = []
        while True:
            if len(self.buf) < 2:
                return out
            b0, b1 = self.buf[0], self.buf[1]
            fin, op, masked, n = b0 & 0x80, b0 & 0x0F, b1 & 0x80, b1 & 0x7F
            pos = 2
            if n == 126:
                if len(self.buf) < 4:
                    return out
                n = struct.unpack("!H", self.buf[2:4])[0]
                pos = 4
            elif n == 127:
                if len(self.buf) < 10:
                    return out
                n = struct.unpack("!Q", self.buf[2:10])[0]
                pos = 10
            if n > MAX_MESSAGE:
                raise ValueError("frame too large")
            if not masked and self.require_mask:
                raise ValueError("unmasked client frame")
            if op >= 0x8 and (not fin or n > 125):
                raise ValueError("bad control frame")
            mask = b""
            if masked:
                if len(self.buf) < pos + 4:
                    return out
                mask = bytes(self.buf[pos:pos + 4])
                pos += 4
            if len(self.buf) < pos + n:
                return out
            payload = bytes(self.buf[pos:pos + n])
            del self.buf[:pos + n]
            if masked:
                payload = bytes(c ^ mask[i & 3] for i, c in enumerate(payload))
            if op >= 0x8:                      # control frame
                out.append((op, payload))
                continue
            if op == 0x0:                      # continuation
                if self.frag_op is None:
                    raise ValueError("unexpected continuation")
                self.frag_len += len(payload)
                if self.frag_len > MAX_MESSAGE:
                    raise ValueError("message too large")
                self.frag.append(payload)
                if fin:
                    out.append((self.frag_op, b"".join(self.frag)))
                    self.frag_op, self.frag, self.frag_len = None, [], 0
                continue
            if self.frag_op is not None:
                raise ValueError("new data frame inside a fragmented message")
            if fin:
                out.append((op, payload))
            else:
                self.frag_op, self.frag, self.frag_len = op, [payload], len(payload)


class RFC6455Protocol(asyncio.Protocol):
    def __init__(self, config, server_state, app_state: Dict[str, Any], _loop=None) -> None:
        if not config.loaded:
            config.load()
        self.config = config
        self.app = config.loaded_app
        self.app_state = app_state
        self.server_state = server_state
        self.loop = _loop or asyncio.get_event_loop()
        self.transport: Optional[asyncio.Transport] = None
        self.head = bytearray()
        self.handshake_done = False
        self.accepted = False
        self.closed = False
        self.parser = FrameParser()
        # bounded: the /clock handler never reads; a flooding client is paused, then failed
        self.queue: "asyncio.Queue[Dict[str, Any]]" = asyncio.Queue()
        self.reading_paused = False
        self.scope: Dict[str, Any] = {}
        self.key = b""
        self.task: Optional[asyncio.Task] = None

    # ------------------------------------------------------------------ asyncio.Protocol
    def connection_made(self, transport) -> None:
        self.transport = transport
        self.server_state.connections.add(self)

    def connection_lost(self, exc) -> None:
        self.server_state.connections.discard(self)
        if not self.closed:
            self.closed = True
            self.queue.put_nowait({"type": "websocket.disconnect", "code": 1006})

    def shutdown(self) -> None:   # called by uvicorn on server shutdown
        if not self.closed and self.transport is not None:
            self._write_frame(0x8, struct.pack("!H", 1012))
            self.transport.close()

    def data_received(self, data: bytes) -> None:
        if not self.handshake_done:
            self.head += data
            end = self.head.find(b"\r\n\r\n")
            if end < 0:
                if len(self.head) > MAX_HANDSHAKE:
                    self._reject(431)
                return
            if end > MAX_HANDSHAKE:
                self._reject(431)
                return
            rest = bytes(self.head[end + 4:])
            self._start(bytes(self.head[:end]))
            data = rest
            if not data:
                return
        try:
            msgs = self.parser.feed(data)
        except ValueError:
            self._fail(1002)
            return
        for op, payload in msgs:
            if op in (0x1, 0x2) and self._data_queued() >= MAX_QUEUED:
                self._fail(1008)               # policy violation: the app is not reading
                return
            if op == 0x1:
                self.queue.put_nowait({"type": "websocket.receive", "text": payload.decode("utf-8", "replace")})
            elif op == 0x2:
                self.queue.put_nowait({"type": "websocket.receive", "bytes": payload})
            elif op == 0x9:
                self._write_frame(0xA, payload)
            elif op == 0x8:
                code = struct.unpack("!H", payload[:2])[0] if len(payload) >= 2 else 1005
                if not self.closed:
                    self._write_frame(0x8, payload[:2])
                    self.closed = True
                    self.queue.put_nowait({"type": "websocket.disconnect", "code": code})
                    self.transport.close()

    # ------------------------------------------------------------------ handshake / ASGI
    def _start(self, head: bytes) -> None:
        self.handshake_done = True
        lines = head.split(b"\r\n")
        method, target, _ = lines[0].split(b" ", 2)
        headers = []
        for ln in lines[1:]:
            if b":" in ln:
                k, v = ln.split(b":", 1)
                headers.append((k.strip().lower(), v.strip()))
        hd = dict(headers)
        self.key = hd.get(b"sec-websocket-key", b"")
        path, _, query = target.partition(b"?")
        client = self.transport.get_extra_info("peername") if self.transport else None
        server = self.transport.get_extra_info("sockname") if self.transport else None
        proto = hd.get(b"sec-websocket-protocol", b"")
        self.scope = {
            "type": "websocket", "asgi": {"version": "3.0", "spec_version": "2.3"}, "http_version": "1.1",
            "scheme": "ws", "server": tuple(server[:2]) if server else None,
            "client": tuple(client[:2]) if client else None, "root_path": self.config.root_path,
            "path": unquote(path.decode("ascii", "replace")), "raw_path": path, "query_string": query,
            "headers": headers, "subprotocols": [p.strip() for p in proto.decode().split(",") if p.strip()],
            "state": self.app_state.copy(),
        }
        self.queue.put_nowait({"type": "websocket.connect"})
        self.task = self.loop.create_task(self._run())

    async def _run(self) -> None:
        try:
            await self.app(self.scope, self._receive, self._send)
        except Exception:  # noqa: BLE001
            log.exception("websocket application error")
            if not self.accepted:
                self._reject(500)
            else:
                self._fail(1011)
        finally:
            if not self.closed and self.transport is not None:
                if self.accepted:
                    self._write_frame(0x8, struct.pack("!H", 1000))
                self.closed = True
                self.transport.close()

    async def _receive(self) -> Dict[str, Any]:
        msg = await self.queue.get()
        if self.reading_paused and self.queue.qsize() < MAX_QUEUED // 4 and self.transport is not None \
                and not self.transport.is_closing():
            self.transport.resume_reading()
            self.reading_paused = False
        return msg

    async def _send(self, message: Dict[str, Any]) -> None:
        t = message["type"]
        if self.transport is None or self.transport.is_closing():
            if t in ("websocket.send", "websocket.accept"):
                raise RuntimeError("websocket closed")   # starlette maps this to a disconnect
            return
        if t == "websocket.accept":
            extra = b""
            if message.get("subprotocol"):
                extra += b"Sec-WebSocket-Protocol: " + message["subprotocol"].encode() + b"\r\n"
            for k, v in message.get("headers") or []:
                extra += k + b": " + v + b"\r\n"
            self.transport.write(b"HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                                 b"Sec-WebSocket-Accept: " + accept_key(self.key) + b"\r\n" + extra + b"\r\n")
            self.accepted = True
        elif t == "websocket.send":
            if message.get("text") is not None:
                self._write_frame(0x1, message["text"].encode())
            else:
                self._write_frame(0x2, message.get("bytes") or b"")
        elif t == "websocket.close":
            if not self.accepted:
                self._reject(403)
                return
            code = int(message.get("code", 1000))
            reason = (message.get("reason") or "").encode()[:120]
            self._write_frame(0x8, struct.pack("!H", code) + reason)
            self.closed = True
            self.transport.close()

    # ------------------------------------------------------------------ helpers
    def _data_queued(self) -> int:
        n = self.queue.qsize()
        if n >= MAX_QUEUED // 2 and not self.reading_paused and self.transport is not None:
            self.transport.pause_reading()     # back-pressure first; resumed as the app reads
            self.reading_paused = True
        return n

    def _write_frame(self, op: int, payload: bytes) -> None:
        if self.transport is not None and not self.transport.is_closing():
            self.transport.write(encode_frame(op, payload))

    def _reject(self, status: int) -> None:
        if self.transport is not None and not self.transport.is_closing():
            reason = {403: "Forbidden", 431: "Request Header Fields Too Large", 500: "Internal Server Error"}.get(status, "Error")
            self.transport.write(f"HTTP/1.1 {status} {reason}\r\ncontent-length: 0\r\nconnection: close\r\n\r\n".encode())
            self.closed = True
            self.transport.close()

    def _fail(self, code: int) -> None:
        self._write_frame(0x8, struct.pack("!H", code))
        self.closed = True
        if self.transport is not None:
            self.transport.close()
        self.queue.put_nowait({"type": "websocket.disconnect", "code": code})
