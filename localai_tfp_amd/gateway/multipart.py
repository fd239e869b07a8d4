"""multipart/form-data and urlencoded form parsing (python-multipart is not available here)."""
from __future__ import annotations

import io
import re
import urllib.parse

_DISP = re.compile(r'(\w+)="((?:[^"\\]|\\.)*)"|(\w+)=([^;\s]+)')


class UploadedFile:
    def __init__(self, filename: str, data: bytes, content_type: str = ""):
        self.filename, self.data, self.content_type = filename, data, content_type
        self.file = io.BytesIO(data)

    async def read(self) -> bytes:
        return self.data


def _params(header_value: str) -> dict:
    out = {}
    for m in _DISP.finditer(header_value):
        if m.group(1):
            out[m.group(1).lower()] = m.group(2).replace('\\"', '"')
        else:
            out[m.group(3).lower()] = m.group(4)
    return out


def parse_multipart(body: bytes, content_type: str) -> dict:
    b = _params(content_type).get("boundary")
    if not b:
        raise ValueError("multipart boundary missing")
    delim = b"--" + b.encode()
    out: dict = {}
    for part in body.split(delim)[1:]:
        if part.startswith(b"--"):
            break
        part = part[2:] if part.startswith(b"\r\n") else part
        head, sep, data = part.partition(b"\r\n\r\n")
        if not sep:
            continue
        if data.endswith(b"\r\n"):
            data = data[:-2]
        headers = {}
        for line in head.decode("utf-8", "replace").split("\r\n"):
            k, _, v = line.partition(":")
            headers[k.strip().lower()] = v.strip()
        disp = _params(headers.get("content-disposition", ""))
        name = disp.get("name", "")
        if "filename" in disp:
            out[name] = UploadedFile(disp["filename"], data, headers.get("content-type", ""))
        else:
            out[name] = data.decode("utf-8", "replace")
    return out


async def read_form(request) -> dict:
    ct = request.headers.get("content-type", "")
    body = await request.body()
    if ct.startswith("multipart/form-data"):
        return parse_multipart(body, ct)
    if ct.startswith("application/x-www-form-urlencoded"):
        return {k: v[-1] for k, v in urllib.parse.parse_qs(body.decode(), keep_blank_values=True).items()}
    if ct.startswith("application/json"):
        import json
        return json.loads(body or b"{}")
    return {}
