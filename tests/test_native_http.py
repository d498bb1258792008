"""Native HTTP front end (CPU backend): wire-level parity with FastAPI, HTTP/1.1 edge cases, load."""
import json
import os
import re
import socket
import struct
import threading
import time

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from conftest import FIXTURES
from test_contract import assert_same_body

GOLDEN = json.loads((FIXTURES / "reference_contract.json").read_text())
NAMES = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
A1 = b'{"sepal_length":5.1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}'


@pytest.fixture(params=[(0, 0, 0), (200, 0, 0), (0, 20, 0), (0, 3, 1)], ids=["block", "spin", "waitspin", "idlegate"])
def server(iris_cwd, request):
    """Blocking IO threads; busy-polling IO threads + spinning batcher / completer (the completion
    hand-off then skips the eventfd); IO threads that watch for their rows' hand-off for a bounded
    while before blocking (io_wait_spin_us); the idle-engine path only while one connection is open
    (idle_max_conns)."""
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    spin, wait_spin, idle_max = request.param
    srv = NativeServer(Config.from_env(port=0, device="cpu", io_threads=2, io_spin_us=spin, spin_us=spin,
                                       io_wait_spin_us=wait_spin, idle_max_conns=idle_max)).start()
    yield srv
    srv.stop()


def raw(port, data: bytes, n_responses=1, timeout=5.0) -> list:
    """Send raw bytes, read n complete responses -> [(status, headers, body)]."""
    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    s.sendall(data)
    buf = b""
    out = []
    while len(out) < n_responses:
        while b"\r\n\r\n" not in buf:
            chunk = s.recv(65536)
            if not chunk:
                s.close()
                return out
            buf += chunk
        head, rest = buf.split(b"\r\n\r\n", 1)
        lines = head.decode("latin-1").split("\r\n")
        status = int(lines[0].split()[1])
        headers = {k.lower(): v.strip() for k, v in (l.split(":", 1) for l in lines[1:])}
        if status == 100:
            buf = rest
            continue
        n = int(headers.get("content-length", 0))
        while len(rest) < n:
            rest += s.recv(65536)
        out.append((status, headers, rest[:n]))
        buf = rest[n:]
    s.close()
    return out


def post(body: bytes, ctype=b"application/json", extra=b"") -> bytes:
    h = b"POST /predict HTTP/1.1\r\nHost: t\r\n"
    if ctype is not None:
        h += b"Content-Type: " + ctype + b"\r\n"
    return h + extra + b"Content-Length: %d\r\n\r\n" % len(body) + body


@pytest.mark.parametrize("case", [c for c in GOLDEN if c["name"] != "A18"], ids=lambda c: c["name"])
def test_golden_over_the_wire(server, case):
    req = case["request"]
    if req["method"] == "GET":
        data = f"GET {req['path']} HTTP/1.1\r\nHost: t\r\n\r\n".encode()
    else:
        body = req["content"].encode() if "content" in req else json.dumps(req["json"]).encode()
        ctype = req.get("headers", {}).get("content-type", "application/json")
        data = post(body, ctype.encode())
    (status, headers, body), = raw(server.port, data)
    assert status == case["status"]
    assert headers["content-type"] == case["content_type"]
    assert_same_body(body.decode(), case["body"], status)
    assert headers["server"] == "uvicorn" and "date" in headers


def test_fast_path_is_taken(server):
    raw(server.port, post(A1))
    assert server.http.stats()["fast"] >= 1


def test_keepalive_and_pipelining(server):
    reqs = post(A1) * 5 + b"GET /nope HTTP/1.1\r\nHost: t\r\n\r\n" + post(A1)
    res = raw(server.port, reqs, n_responses=7)
    assert [r[0] for r in res] == [200] * 5 + [404, 200]


def test_chunked_and_expect_continue(server):
    body = A1
    chunked = b"%x\r\n%s\r\n%x\r\n%s\r\n0\r\n\r\n" % (10, body[:10], len(body) - 10, body[10:])
    data = (b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\n"
            b"Transfer-Encoding: chunked\r\n\r\n" + chunked)
    (status, _, b), = raw(server.port, data)
    assert status == 200 and json.loads(b)["prediction"] == "Iris-setosa"
    (status, _, _), = raw(server.port, post(A1, extra=b"Expect: 100-continue\r\n"))
    assert status == 200


def test_http10_closes(server):
    s = socket.create_connection(("127.0.0.1", server.port))
    s.sendall(b"POST /predict HTTP/1.0\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
              % (len(A1), A1))
    data = b""
    while True:
        c = s.recv(4096)
        if not c:
            break
        data += c
    assert data.startswith(b"HTTP/1.1 200") and b"connection: close" in data


def test_malformed_requests(server):
    (status, _, _), = raw(server.port, b"GARBAGE\r\n\r\n")
    assert status == 400
    (status, _, _), = raw(server.port, b"POST /predict HTTP/1.1\r\nContent-Length: x\r\n\r\n")
    assert status == 400
    (status, _, _), = raw(server.port, b"POST /predict HTTP/1.1\r\nContent-Length: 999999999999\r\n\r\n")
    assert status == 413


def test_files_via_slow_path(server):
    from mlapi_amd.api.multipart import encode_multipart

    body, ctype = encode_multipart({"token": "abc"}, {"file": ("x.csv", b"c\n0.5\n", "text/csv")})
    data = (b"POST /files/ HTTP/1.1\r\nHost: t\r\nContent-Type: " + ctype.encode() +
            b"\r\nContent-Length: %d\r\n\r\n" % len(body) + body)
    (status, _, b), = raw(server.port, data)
    assert status == 200 and json.loads(b) == {"file": {"c": {"0": 0.5}}, "token": "abc"}


def test_loadgen_concurrency_and_batching(server, native):
    req = post(A1).decode()
    lg = native.Loadgen("127.0.0.1", server.port, req, 32, 2)
    r = lg.run(100, True)
    lg.close()
    assert r["status_counts"] == {200: 3200} and r["failed"] == 0
    assert len(r["latencies_ns"]) == 3200


def test_client_disconnect_mid_request(server):
    s = socket.create_connection(("127.0.0.1", server.port))
    s.sendall(post(A1)[:-5])
    s.close()
    time.sleep(0.05)
    (status, _, _), = raw(server.port, post(A1))
    assert status == 200


# ------------------------------------------------------------------ fast-path parser units
def _parse(native, body: str):
    return native.parse_predict_body(body, NAMES)


def test_parser_accepts_plain_numbers(native):
    assert _parse(native, '{"sepal_length":5.1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}') == \
        [5.1, 3.5, 1.4, 0.2]
    assert _parse(native, ' { "petal_width" : -0e0 , "sepal_length":1E2,"sepal_width":0,"petal_length":12345678901234567890 } ') \
        == [100.0, 0.0, 12345678901234567890.0, -0.0]
    assert _parse(native, '{"x":{"a":[1,"}",{"b":null}]},"sepal_length":1,"sepal_width":2,"petal_length":3,'
                          '"petal_width":4,"y":true}') == [1, 2, 3, 4]


@pytest.mark.parametrize("tok", [
    "0", "-0", "0.0", "-0.0", "7", "1234567", "12345678", "123456789", "0.1234567", "0.12345678",
    "1234567.1234567", "1234567.12345678", "9999999.9999999", "5.", "-", "-a", "01", "-01", "00.5", "1.e5",
    "1.5e3", "1.5E-3", "2e0", "0e5", "1234567e-7", ".5", "+1", "1.2.3", "1..2", "3.14159", "-2.5", "100",
])
def test_parser_swar_numbers_match_json(native, tok):
    """Numbers followed by >= 24 more bytes take the 8-byte-at-a-time (SWAR) path of
    csrc/http/json_body.cpp: every token parses to exactly float(tok) when json.loads accepts it,
    and is refused (slow path) when it does not - including runs of exactly 7 / 8 digits."""
    names = ["a", "b"]
    body = '{"a":' + tok + ', "b": 1, "padding_padding_padding": 0}'
    try:
        want = json.loads(body)["a"]
        ok = isinstance(want, (int, float)) and not isinstance(want, bool)
    except ValueError:
        ok = False
    got = native.parse_predict_body(body, names)
    if not ok:
        assert got is None, tok
    else:
        assert got is not None, tok
        assert struct.pack("<d", got[0]) == struct.pack("<d", float(want)), tok
        assert got[1] == 1.0


def test_parser_key_prefixes_and_unclean_names(native):
    """The schema-order key match compares name + closing quote: a name that is a prefix of the
    next key must not match it, and a name JSON can only spell escaped never matches (slow path)."""
    assert native.parse_predict_body('{"f10":2,"f1":1}', ["f1", "f10"]) == [1.0, 2.0]
    assert native.parse_predict_body('{"f1":1,"f10":2}', ["f1", "f10"]) == [1.0, 2.0]
    assert native.parse_predict_body('{"f1" :1, "f10":2 ,"f1":3}', ["f1", "f10"]) == [3.0, 2.0]
    assert native.parse_predict_body('{"f1":1,"a\\"b":3}', ["f1", 'a"b']) is None
    assert native.parse_predict_body('{"f1":1,"a"b":3}', ["f1", 'a"b']) is None


@pytest.mark.parametrize("body", [
    '{"sepal_length":"5.1","sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',  # string -> pydantic coerces
    '{"sepal_length":NaN,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"sepal_length":1e400,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',  # inf
    '{"sepal_length":01,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"sepal_length":1.,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"sepal_length":null,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"sepal_length":true,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"sepal_length":1,"sepal_width":3.5,"petal_length":1.4}',
    '{"sepal\\u005flength":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '[1,2,3,4]', 'hello', '', '{"sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2} x',
    '{"sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2,}',
    # extra values json.loads rejects: the fast path must not answer 200 for them
    '{"x":1..2e-,"sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"x":-,"sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"x":"\\q","sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"x":"\\u12","sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"x":1.5e,"sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"x":--1,"sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"x":01,"sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"x":"\u00e9","sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
])
def test_parser_delegates_everything_else(native, body):
    assert _parse(native, body) is None


@pytest.mark.parametrize("body", [
    '{"x":"a\\"b\\\\c\\/\\b\\f\\n\\r\\t\\u00e9","sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
    '{"x":[1e400,-0.5E-3,0,{"y":[]}],"sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
])
def test_parser_accepts_valid_extras(native, body):
    json.loads(body)  # the reference accepts these bodies too
    assert _parse(native, body) == [1, 3.5, 1.4, 0.2]


def test_invalid_extra_value_gets_fastapi_422(server):
    body = b'{"x":1..2e-,"sepal_length":1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}'
    (status, _, b), = raw(server.port, post(body))
    assert status == 422 and json.loads(b)["detail"][0]["type"] == "json_invalid"


@pytest.mark.parametrize("size", [b"ffffffffffffffff", b"-1", b"10000000000000000", b"0x10", b"zz"])
def test_chunked_size_overflow_is_rejected(server, size):
    """a huge / negative / malformed chunk size once aborted the process."""
    data = (b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\n"
            b"Transfer-Encoding: chunked\r\n\r\n1\r\n{\r\n" + size + b"\r\nxxxx")
    res = raw(server.port, data)
    assert res and res[0][0] in (400, 413)
    (status, _, _), = raw(server.port, post(A1))  # the server is still alive
    assert status == 200


def test_chunk_without_crlf_terminator_is_rejected(server):
    data = (b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\n"
            b"Transfer-Encoding: chunked\r\n\r\n2\r\n{}XX0\r\n\r\n")
    (status, _, _), = raw(server.port, data)
    assert status == 400


def test_pipelined_flood_while_waiting_is_served_in_order(iris_cwd):
    """A client that keeps writing while its first request is in the engine: the server stops
    reading past pipeline_cap (bounded memory) and resumes once the response is out."""
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    srv = NativeServer(Config.from_env(port=0, device="cpu", io_threads=1, delay_us=5000)).start()
    try:
        n = 200  # 200 x 8 KB = 1.6 MB pipelined behind a 5 ms batch: > the 1 MiB pipeline cap
        body = A1[:-1] + b',"pad":"' + b"a" * 8192 + b'"}'
        res = raw(srv.port, post(body) * n, n_responses=n, timeout=60)
        assert len(res) == n and all(r[0] == 200 for r in res)
        assert srv.http.stats()["fast"] >= n
    finally:
        srv.stop()


def test_access_log_uvicorn_format(iris_cwd, tmp_path):
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    r, w = os.pipe()
    srv = NativeServer(Config.from_env(port=0, device="cpu", io_threads=1, access_log=True), access_log_fd=w)
    srv.start()
    try:
        raw(srv.port, post(A1))
        raw(srv.port, b"GET /nope HTTP/1.1\r\nHost: t\r\n\r\n")
        time.sleep(0.5)
        os.set_blocking(r, False)
        text = os.read(r, 65536).decode()
    finally:
        srv.stop()
        os.close(r)
        os.close(w)
    lines = text.strip().splitlines()
    assert re.match(r'^INFO:     127\.0\.0\.1:\d+ - "POST /predict HTTP/1\.1" 200 OK$', lines[0]), lines
    assert re.match(r'^INFO:     127\.0\.0\.1:\d+ - "GET /nope HTTP/1\.1" 404 Not Found$', lines[1]), lines


@settings(max_examples=300, deadline=None)
@given(st.lists(st.floats(allow_nan=False, allow_infinity=False), min_size=4, max_size=4),
       st.dictionaries(st.text(min_size=1, max_size=5), st.integers() | st.text(max_size=5) | st.none(), max_size=3))
def test_parser_matches_json_loads(native, vals, extra):
    d = dict(extra)
    d.update(zip(NAMES, vals))
    body = json.dumps(d)
    got = _parse(native, body)
    if got is None:  # only acceptable when an extra key needed escapes (delegated, still correct)
        assert "\\" in body
    else:
        assert got == [json.loads(body)[n] for n in NAMES]


@settings(max_examples=2000, deadline=None)
@given(st.floats(allow_nan=False, allow_infinity=False))
def test_float_repr_matches_python(native, v):
    assert native.py_float_repr(v) == repr(v) == json.dumps(v)


def test_fast_number_path_matches_python_float(native):
    """The parser's Clinger fast path (<= 15 significant digits, |10^e| <= 22) and its strtod
    fallback both give Python's float() bit for bit, over tokens of every shape the wide-model
    bodies and the reference's clients send."""
    import random
    import struct

    rng = random.Random(12)
    toks = ["0", "-0", "0.0", "-0.0", "1", "-1", "5.1", "3.5", "1e22", "1e23", "1e-22", "1e-23", "9007199254740993",
            "123456789012345", "1234567890123456", "0.1", "0.30000000000000004", "1.7976931348623157e308",
            "2.2250738585072014e-308", "4.9e-324", "1E+2", "1e-0", "0.000000000000000000001", "100000000000000000000000",
            "123.456e-5", "-9.87654321012345e10"]
    for _ in range(3000):
        kind = rng.randrange(4)
        if kind == 0:
            toks.append(repr(rng.gauss(0, 1)))
        elif kind == 1:
            toks.append(f"{rng.uniform(-1e4, 1e4):.{rng.randrange(0, 8)}f}")
        elif kind == 2:
            toks.append(f"{rng.randrange(1, 10**rng.randrange(1, 18))}e{rng.randrange(-30, 30)}")
        else:
            toks.append(f"{rng.choice(['', '-'])}{rng.randrange(0, 10**6)}.{rng.randrange(0, 10**rng.randrange(1, 12))}")
    names = [f"f{i}" for i in range(len(toks))]
    body = "{" + ",".join(f'"{n}":{t}' for n, t in zip(names, toks)) + "}"
    got = native.parse_predict_body(body, names)
    assert got is not None
    for t, g in zip(toks, got):  # the FastAPI oracle: json.loads (an integer literal is an int), then float
        assert struct.pack("<d", g) == struct.pack("<d", float(json.loads(t))), t


def test_idle_engine_fast_path_cpu_backend(iris_cwd):
    """One client at a time: the IO thread runs the row itself (Engine::run_idle, here the float64
    oracle of the CPU backend), bodies identical to the queued path; under concurrency the batcher
    still coalesces."""
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    rng = np.random.default_rng(3)
    bodies = [json.dumps(dict(zip(NAMES, map(float, np.round(r, 1))))).encode() for r in
              rng.normal([5.8, 3.0, 3.8, 1.2], [0.8, 0.4, 1.8, 0.8], (60, 4))]
    out = {}
    for rows in (8, 0):
        srv = NativeServer(Config.from_env(port=0, device="cpu", io_threads=2, idle_inline_rows=rows)).start()
        try:
            s = socket.create_connection(("127.0.0.1", srv.port), timeout=5)
            got = []
            for b in bodies:
                s.sendall(post(b))
                buf = b""
                while not buf.endswith(b"}"):
                    buf += s.recv(4096)
                got.append(buf.split(b"\r\n\r\n", 1)[1])
            s.close()
            st = srv.runtime.handle.stats()
            assert (st["idle_batches"] >= 50) if rows else st["idle_batches"] == 0, st
            out[rows] = got
        finally:
            srv.stop()
    assert out[8] == out[0]


def test_metrics_expose_http_latency_stages_and_rejections(iris_cwd):
    """/metrics on the native server: the server-side HTTP latency histogram, the per-stage IO
    thread clock, queue wait, backpressure rejections and the serving dtypes."""
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    srv = NativeServer(Config.from_env(port=0, device="cpu", io_threads=2)).start()
    try:
        for _ in range(50):
            assert raw(srv.port, b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\n"
                                 b"Content-Length: %d\r\n\r\n%s" % (len(A1), A1))[0][0] == 200
        time.sleep(0.3)  # IO threads publish their clocks once per loop
        st = srv.http.stats()
        assert st["http_latency_count"] >= 50 and sum(st["http_latency_hist_us_pow2"]) == st["http_latency_count"]
        assert st["stage_ns"]["parse"] > 0 and st["stage_ns"]["send"] > 0 and st["stage_ns"]["recv"] > 0
        (_, _, body), = raw(srv.port, b"GET /metrics HTTP/1.1\r\nHost: t\r\n\r\n")
        m = body.decode()
        for name in ('mlapi_http_request_duration_seconds_bucket{rank="0",backend="cpu",le="+Inf"}',
                     "mlapi_http_request_duration_seconds_count", 'mlapi_server_stage_seconds_total{rank="0",'
                     'backend="cpu",stage="parse"}', "mlapi_requests_rejected_total", "mlapi_queue_wait_seconds_total",
                     'mlapi_serving_dtype_info{rank="0",backend="cpu",small="f64",wide="f64"} 1'):
            assert name in m, name
    finally:
        srv.stop()


def test_fast_parser_matches_full_parser_on_header_variants(server):
    """The zero-allocation fast path and the full parser answer header variants identically:
    case-insensitive names, duplicate content-type (last wins), query string, Connection: close,
    and HTTP/1.0 / chunked / Expect requests (full parser) all give the same 200 body."""
    pre = b"POST /predict?x=1 HTTP/1.1\r\nHOST: t\r\ncontent-TYPE:  application/json ; charset=utf-8 \r\nX-A: b\r\n"
    r1 = raw(server.port, pre + b"CONTENT-LENGTH: %d\r\n\r\n%s" % (len(A1), A1))
    r2 = raw(server.port, b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked"
                          b"\r\n\r\n%x\r\n%s\r\n0\r\n\r\n" % (len(A1), A1))
    r3 = raw(server.port, b"POST /predict HTTP/1.0\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
             % (len(A1), A1))
    r4 = raw(server.port, b"POST /predict HTTP/1.1\r\nContent-Type: application/json\r\nConnection: Close\r\n"
                          b"Content-Length: %d\r\n\r\n%s" % (len(A1), A1))
    assert r1[0][0] == r2[0][0] == r3[0][0] == r4[0][0] == 200
    assert r1[0][2] == r2[0][2] == r3[0][2] == r4[0][2]
    assert r4[0][1].get("connection") == "close"
    # duplicate Content-Type: FastAPI reads the FIRST one (Starlette headers[...]); text/plain first -> 422
    r5 = raw(server.port, b"POST /predict HTTP/1.1\r\nContent-Type: text/plain\r\nContent-Type: application/json\r\n"
                          b"Content-Length: %d\r\n\r\n%s" % (len(A1), A1))
    assert r5[0][0] == 422
    r6 = raw(server.port, b"POST /predict HTTP/1.1\r\nContent-Type: application/json\r\nContent-Type: text/plain\r\n"
                          b"Content-Length: %d\r\n\r\n%s" % (len(A1), A1))
    assert r6[0][0] == 200 and r6[0][2] == r1[0][2]
