"""Closed-loop HTTP load generator for /v1/chat/completions (SSE streaming).

`--concurrency` virtual users each send a chat request, consume the SSE stream, record
(t_send, t_first_content, t_end, completion_tokens) with time.monotonic() (system-wide clock on
Linux, so the numbers line up with the server process), and immediately send the next request.
Runs until SIGTERM/SIGINT or `--duration`, then writes all records as JSON to `--out`.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import random
import signal
import time

WORDS = ["the", "model", "serves", "tokens", "fast", "on", "MI355X", "with", "paged", "attention", "and",
         "hipGraph", "decode", "kernels", "for", "every", "request", "in", "batch", "xGMI"]


async def one(session, url, body, rec, stop):
    t0 = time.monotonic()
    r = {"t_send": t0, "t_first": None, "t_end": None, "tokens": 0, "chunks": 0, "ok": False, "t_chunks": []}
    try:
        async with session.post(url, json=body) as resp:
            buf = b""
            async for chunk in resp.content.iter_any():
                buf += chunk
                while b"\n\n" in buf:
                    ev, buf = buf.split(b"\n\n", 1)
                    if not ev.startswith(b"data: "):
                        continue
                    payload = ev[6:]
                    if payload == b"[DONE]":
                        r["ok"] = True
                        continue
                    j = json.loads(payload)
                    ch = (j.get("choices") or [{}])
                    d = ch[0].get("delta") or {} if ch else {}
                    if d.get("content"):
                        now = time.monotonic()
                        r["chunks"] += 1
                        r["t_chunks"].append(now)
                        if r["t_first"] is None:
                            r["t_first"] = now
                    u = j.get("usage")
                    if u:
                        r["tokens"] = u.get("completion_tokens", r["tokens"])
    except (asyncio.CancelledError, Exception) as ex:  # noqa: BLE001 - record and move on
        r["error"] = type(ex).__name__
    r["t_end"] = time.monotonic()
    rec.append(r)


async def user(session, url, mk_body, rec, stop: asyncio.Event, first_len: int | None = None):
    n = 0
    while not stop.is_set():
        body = mk_body()
        if n == 0 and first_len:
            body["max_tokens"] = first_len
        n += 1
        await one(session, url, body, rec, stop)


async def run(a):
    import aiohttp
    rng = random.Random(a.seed)
    url = a.url.rstrip("/") + "/v1/chat/completions"

    def mk_body():
        if a.prompt_words:  # subword tokenizer: the caller sized the word count to the token budget
            content = " ".join(rng.choice(WORDS) for _ in range(a.prompt_words))
        else:  # byte tokenizer: one token per character
            n_words = max(1, a.prompt_chars // 6)
            content = " ".join(rng.choice(WORDS) for _ in range(n_words))[: a.prompt_chars]
        body = {"model": a.model, "stream": True, "max_tokens": a.gen_len, "temperature": a.temperature,
                "ignore_eos": True, "messages": [{"role": "user", "content": content}]}
        if a.frequency_penalty:
            body["frequency_penalty"] = a.frequency_penalty
        if a.json:
            body["response_format"] = {"type": "json_object"}
        if a.top_k is not None:
            body["top_k"] = a.top_k
        if a.top_p is not None:
            body["top_p"] = a.top_p
        return body
    rec: list = []
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for s in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(s, stop.set)
    conn = aiohttp.TCPConnector(limit=0, force_close=False)
    timeout = aiohttp.ClientTimeout(total=None, sock_read=600)
    async with aiohttp.ClientSession(connector=conn, timeout=timeout) as session:
        # --stagger: user i's first request asks for ceil(gen_len * (i + 1) / concurrency) tokens, so
        # completions (and re-arrivals) are spread evenly from the start: the server reaches the
        # stationary continuous-batching mix (decode rows + arriving prefill chunks) after about
        # one generation length instead of oscillating in lock-step waves.
        C = a.concurrency
        firsts = [(-(-a.gen_len * (i + 1) // C) if a.stagger else None) for i in range(C)]
        tasks = [asyncio.ensure_future(user(session, url, mk_body, rec, stop, firsts[i])) for i in range(C)]
        if a.duration:
            try:
                await asyncio.wait_for(stop.wait(), a.duration)
            except asyncio.TimeoutError:
                stop.set()
        else:
            await stop.wait()
        for t in tasks:
            t.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)
    with open(a.out, "w") as f:
        json.dump(rec, f)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", required=True)
    ap.add_argument("--model", required=True)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--prompt-chars", type=int, default=220)
    ap.add_argument("--gen-len", type=int, default=256)
    ap.add_argument("--prompt-words", type=int, default=0, help="prompt of N words (overrides --prompt-chars)")
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--top-k", type=int, default=None)
    ap.add_argument("--top-p", type=float, default=None)
    ap.add_argument("--frequency-penalty", type=float, default=0.0)
    ap.add_argument("--json", action="store_true", help="response_format json_object (grammar-constrained)")
    ap.add_argument("--duration", type=float, default=0.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--stagger", action="store_true", help="spread the first requests' lengths evenly")
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    asyncio.run(run(a))


if __name__ == "__main__":
    main()
