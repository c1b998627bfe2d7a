"""The in-tree RFC 6455 protocol used to serve /clock under uvicorn (no websockets/wsproto on
the image): handshake key, frame codec, and a live uvicorn round trip of the clock message."""
import asyncio
import base64
import os
import socket
import struct
import threading
import time

import numpy as np
import pytest

from cassmantle_amd.api.wsproto import FrameParser, accept_key, encode_frame


def _mask(op, payload, fin=True):
    m = os.urandom(4)
    b0 = (0x80 if fin else 0) | op
    n = len(payload)
    head = bytes([b0, 0x80 | n]) if n < 126 else struct.pack("!BBH", b0, 0x80 | 126, n)
    return head + m + bytes(c ^ m[i % 4] for i, c in enumerate(payload))


def test_accept_key_rfc_example():
    assert accept_key(b"dGhlIHNhbXBsZSBub25jZQ==") == b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo="


def test_frame_codec_fragmented_and_control():
    p = FrameParser()
    data = _mask(0x1, b"hel", fin=False) + _mask(0x9, b"pi") + _mask(0x0, b"lo" * 100)
    # feed byte by byte: the parser must be incremental
    out = []
    for i in range(len(data)):
        out += p.feed(data[i:i + 1])
    assert out == [(0x9, b"pi"), (0x1, b"hel" + b"lo" * 100)]
    f = encode_frame(0x1, b"x" * 300)
    assert f[1] == 126 and struct.unpack("!H", f[2:4])[0] == 300


def test_live_uvicorn_clock():
    import uvicorn
    from cassmantle_amd.api.app import create_app
    from cassmantle_amd.config import Config
    from cassmantle_amd.game.content import SolidImageGenerator
    from cassmantle_amd.game.service import GameService
    from cassmantle_amd.scoring.batcher import BatchingScorer
    from cassmantle_amd.scoring.wordvec import WordVectorBackend

    cfg = Config()
    cfg.game.clock_period = 0.05
    be = WordVectorBackend(vocab=["a", "b"], vectors=np.eye(2, dtype=np.float32))
    svc = GameService(cfg, BatchingScorer(be, 0.01), image_gen_for_room=lambda r: SolidImageGenerator(32))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    config = uvicorn.Config(create_app(svc, cfg, run_timers=False), host="127.0.0.1", port=port,
                            ws="cassmantle_amd.api.wsproto:RFC6455Protocol", log_level="warning")
    server = uvicorn.Server(config)
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    try:
        for _ in range(100):
            if server.started:
                break
            time.sleep(0.05)
        c = socket.create_connection(("127.0.0.1", port), timeout=5)
        key = base64.b64encode(os.urandom(16)).decode()
        c.sendall(f"GET /clock HTTP/1.1\r\nHost: x\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                  f"Sec-WebSocket-Key: {key}\r\nSec-WebSocket-Version: 13\r\n\r\n".encode())
        buf = b""
        while b"\r\n\r\n" not in buf:
            buf += c.recv(4096)
        head, _, rest = buf.partition(b"\r\n\r\n")
        assert head.startswith(b"HTTP/1.1 101")
        assert accept_key(key.encode()) in head
        p = FrameParser(require_mask=False)    # server frames are unmasked
        msgs = p.feed(rest)
        while not msgs:
            msgs = p.feed(c.recv(4096))
        op, payload = msgs[0]
        assert op == 0x1 and b'"time"' in payload and b'"conns"' in payload
        c.sendall(_mask(0x8, struct.pack("!H", 1000)))
        c.close()
    finally:
        server.should_exit = True
        th.join(timeout=10)


def _unmasked(op, payload, fin=True):
    b0 = (0x80 if fin else 0) | op
    return bytes([b0, len(payload)]) + payload


def test_parser_rejects_protocol_violations():
    from cassmantle_amd.api import wsproto
    with pytest.raises(ValueError):                      # RFC 6455 §5.1: clients must mask
        FrameParser().feed(_unmasked(0x1, b"hi"))
    with pytest.raises(ValueError):                      # fragmented control frame
        FrameParser().feed(_mask(0x9, b"x", fin=False))
    with pytest.raises(ValueError):                      # continuation without a start
        FrameParser().feed(_mask(0x0, b"x"))
    # reassembled message above the cap, although every single frame is small
    p = FrameParser()
    chunk = b"a" * 60000
    p.feed(_mask(0x1, chunk, fin=False))
    with pytest.raises(ValueError):
        for _ in range(wsproto.MAX_MESSAGE // len(chunk) + 1):
            p.feed(_mask(0x0, chunk, fin=False))


class _FakeTransport:
    def __init__(self):
        self.written = b""
        self.closed = False
        self.paused = False

    def write(self, b):
        self.written += b

    def close(self):
        self.closed = True

    def is_closing(self):
        return self.closed

    def pause_reading(self):
        self.paused = True

    def resume_reading(self):
        self.paused = False

    def get_extra_info(self, k):
        return ("127.0.0.1", 1)


def _proto():
    from cassmantle_amd.api.wsproto import RFC6455Protocol

    class Cfg:
        loaded = True
        loaded_app = staticmethod(lambda *a: None)
        root_path = ""

    class State:
        connections = set()

    loop = asyncio.new_event_loop()
    pr = RFC6455Protocol(Cfg(), State(), {}, _loop=loop)
    pr.connection_made(_FakeTransport())
    pr._start = lambda head: setattr(pr, "handshake_done", True)   # no ASGI app needed here
    return pr, loop


def test_protocol_bounds_handshake_queue_and_unmasked():
    from cassmantle_amd.api import wsproto
    pr, loop = _proto()
    pr.data_received(b"GET /clock HTTP/1.1\r\n" + b"X: " + b"y" * (wsproto.MAX_HANDSHAKE + 10))
    assert pr.transport.closed and b" 431 " in pr.transport.written
    loop.close()
    # an application that never reads: reading is paused, then the connection is failed 1008
    pr, loop = _proto()
    pr.data_received(b"GET / HTTP/1.1\r\n\r\n")
    for i in range(wsproto.MAX_QUEUED + 5):
        if pr.closed:
            break
        pr.data_received(_mask(0x1, b"m%d" % i))
    assert pr.transport.paused or pr.closed
    assert pr.closed and struct.pack("!H", 1008) in pr.transport.written
    loop.close()
    # unmasked frame -> close 1002
    pr, loop = _proto()
    pr.data_received(b"GET / HTTP/1.1\r\n\r\n")
    pr.data_received(_unmasked(0x1, b"hi"))
    assert pr.closed and struct.pack("!H", 1002) in pr.transport.written
    loop.close()
