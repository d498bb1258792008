"""multipart/form-data (RFC 7578) and application/x-www-form-urlencoded body parsing.

The reference's `POST /files/` (`main.py:29-30`) declares ``file: bytes = File(...)`` and
``token: str = Form(...)``, which makes FastAPI require the third-party ``python-multipart``
package (`requirements.txt:9`). That package is not available here, so the route reads the raw
body and parses it with this module instead; the OpenAPI schema and the 422 error shapes are
reproduced separately (:mod:`mlapi_amd.api.app`).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple
from urllib.parse import parse_qsl


class MultipartError(ValueError):
    pass


@dataclass
class Part:
    name: str
    data: bytes
    filename: Optional[str] = None
    content_type: Optional[str] = None
    headers: Dict[str, str] = field(default_factory=dict)

    @property
    def is_file(self) -> bool:
        return self.filename is not None


def _parse_header_params(value: str) -> Tuple[str, Dict[str, str]]:
    """'form-data; name="file"; filename="a.csv"' -> ('form-data', {...}). Handles quoted ';'."""
    out: Dict[str, str] = {}
    parts: List[str] = []
    cur, q, esc = [], False, False
    for ch in value:
        if esc:
            cur.append(ch)
            esc = False
        elif ch == "\\" and q:
            esc = True
        elif ch == '"':
            q = not q
            cur.append(ch)
        elif ch == ";" and not q:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    parts.append("".join(cur))
    main = parts[0].strip().lower()
    for p in parts[1:]:
        if "=" not in p:
            continue
        k, v = p.split("=", 1)
        k, v = k.strip().lower(), v.strip()
        if len(v) >= 2 and v[0] == v[-1] == '"':
            v = v[1:-1]
        out[k] = v
    return main, out


def content_type_of(header: Optional[str]) -> Tuple[str, Dict[str, str]]:
    if not header:
        return "", {}
    return _parse_header_params(header)


def parse_multipart(body: bytes, boundary: str) -> List[Part]:
    if not boundary:
        raise MultipartError("missing boundary")
    delim = b"--" + boundary.encode("latin-1")
    parts: List[Part] = []
    pos = body.find(delim)
    if pos < 0:
        raise MultipartError("boundary not found")
    pos += len(delim)
    while True:
        if body[pos:pos + 2] == b"--":
            break  # closing delimiter
        # skip transport padding + CRLF after the delimiter
        eol = body.find(b"\r\n", pos)
        if eol < 0:
            raise MultipartError("truncated part")
        pos = eol + 2
        hend = body.find(b"\r\n\r\n", pos)
        if hend < 0:
            raise MultipartError("truncated part headers")
        headers: Dict[str, str] = {}
        for line in body[pos:hend].split(b"\r\n"):
            if not line:
                continue
            if b":" not in line:
                raise MultipartError("bad part header")
            k, v = line.split(b":", 1)
            headers[k.decode("latin-1").strip().lower()] = v.decode("utf-8", "replace").strip()
        pos = hend + 4
        nxt = body.find(b"\r\n" + delim, pos)
        if nxt < 0:
            raise MultipartError("unterminated part")
        data = body[pos:nxt]
        pos = nxt + 2 + len(delim)
        disp, params = _parse_header_params(headers.get("content-disposition", ""))
        if disp != "form-data" or "name" not in params:
            continue
        parts.append(Part(name=params["name"], data=data, filename=params.get("filename"),
                          content_type=headers.get("content-type"), headers=headers))
    return parts


def parse_form(body: bytes, content_type_header: Optional[str]) -> List[Part]:
    """Starlette ``request.form()`` equivalent: multipart, urlencoded, or empty for anything else."""
    ctype, params = content_type_of(content_type_header)
    if ctype == "multipart/form-data":
        return parse_multipart(body, params.get("boundary", ""))
    if ctype == "application/x-www-form-urlencoded":
        return [Part(name=k, data=v.encode("utf-8"))
                for k, v in parse_qsl(body.decode("latin-1"), keep_blank_values=True)]
    return []


def encode_multipart(fields: Dict[str, str], files: Dict[str, Tuple[str, bytes, str]],
                     boundary: str = "mlapiboundary7MA4YWxkTrZu0gW") -> Tuple[bytes, str]:
    """Client-side helper (tests / load generator): returns (body, content-type header)."""
    out = bytearray()
    for k, v in fields.items():
        out += f'--{boundary}\r\nContent-Disposition: form-data; name="{k}"\r\n\r\n'.encode()
        out += v.encode() + b"\r\n"
    for k, (fname, data, ctype) in files.items():
        out += (f'--{boundary}\r\nContent-Disposition: form-data; name="{k}"; filename="{fname}"\r\n'
                f"Content-Type: {ctype}\r\n\r\n").encode()
        out += data + b"\r\n"
    out += f"--{boundary}--\r\n".encode()
    return bytes(out), f"multipart/form-data; boundary={boundary}"
