"""Block registry: which server serves which layers, and which layers a new server should take.

Reference: the server loop is meant to "choose optimal block ids" against what the swarm already
serves (/root/reference/distributed_llm_inference/server/server.py:7-8), through hivemind's DHT
(imported at server/backend.py:4-7).  Here the swarm's shared state is one small HTTP service:

    POST /claim     {"model", "num_layers", "max_layers", "url"} -> {"start", "end"}
                    picks the range for a new block server and records it at once (under one
                    lock, so servers starting together never pick the same gap)
    POST /announce  {"model", "url", "start", "end", "num_layers", "ttl"}: the server is up
                    (sent again every ttl / 3 as a heartbeat; an entry that misses its ttl is
                    dropped, a claim that never turns ready after ``claim_ttl`` too)
    POST /withdraw  {"url"}
    POST /rebalance {"model", "url", "num_layers", "max_layers"} -> {"move", "start", "end"}
                    should this server move to less-served layers (``rebalance_target``)? A move
                    is recorded at once as the server's new claim, so servers rebalancing
                    together never pile onto the same gap
    GET  /servers?model=M   [{"url", "start", "end", "num_layers", "ready"}]

``distribute registry`` runs it; ``distribute block-serve --registry URL --max-layers N`` claims
a range instead of taking ``--start/--end``, and ``RemoteSequential.from_registry(URL, model)``
builds the client's chain from the registry alone - and re-resolves a failed hop from it
(server/block_server.py failover).  ``block-serve --rebalance-s T`` asks /rebalance every T
seconds while it holds no sessions and moves when the swarm gains from it (the reference's
``should_rebalance`` intent, server/server.py:20).

Trust: the mutating endpoints (/claim, /announce, /withdraw) take a shared token when the
registry is started with one (``distribute registry --token T``; servers pass the same
``--registry-token``): ``Authorization: Bearer T``, else 401.  Without a token anyone who can
reach the registry can announce a URL for a layer range and receive clients' hidden states, so
an open registry belongs on a trusted network only.
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

try:   # module level: FastAPI resolves the (string) annotations of the handlers here
    from fastapi import Request
except ImportError:  # pragma: no cover - clients need no web framework
    Request = None


def _coverage(num_layers: int, served: Sequence[Tuple[int, int]]) -> List[int]:
    cov = [0] * num_layers
    for s, e in served:
        for i in range(max(0, s), min(num_layers, e)):
            cov[i] += 1
    return cov


def choose_range(num_layers: int, max_layers: int,
                 served: Sequence[Tuple[int, int]]) -> Tuple[int, int]:
    """The layer range a new server holding at most ``max_layers`` layers should serve.

    Uncovered layers come first: the first maximal run of layers nobody serves, capped at
    ``max_layers``.  With every layer covered, the window of ``max_layers`` layers with the
    lowest (max coverage, total coverage) -- the least-served part of the model, where one more
    replica adds the most throughput; the lowest start breaks ties."""
    if num_layers <= 0 or max_layers <= 0:
        raise ValueError("num_layers and max_layers must be positive")
    span = min(max_layers, num_layers)
    cov = _coverage(num_layers, served)
    if 0 in cov:
        s = cov.index(0)
        e = s
        while e < num_layers and cov[e] == 0 and e - s < span:
            e += 1
        return s, e
    best = min(range(num_layers - span + 1),
               key=lambda s: (max(cov[s:s + span]), sum(cov[s:s + span]), s))
    return best, best + span


def swarm_score(num_layers: int, served: Sequence[Tuple[int, int]]) -> Tuple[int, int]:
    """How well ``served`` covers the model: every chain passes through every layer, so the
    swarm's throughput is bounded by its least-served layer -- (that coverage, minus the number
    of layers at it); larger is better."""
    cov = _coverage(num_layers, served)
    lo = min(cov)
    return lo, -cov.count(lo)


def rebalance_target(num_layers: int, max_layers: int, others: Sequence[Tuple[int, int]],
                     mine: Tuple[int, int]) -> Optional[Tuple[int, int]]:
    """Where a server now serving ``mine`` should move, given the ranges ``others`` the rest of
    the swarm serves, or None to stay: the window of ``max_layers`` layers (or
    :func:`choose_range`'s pick) with the best :func:`swarm_score`, taken only when it strictly
    beats staying (a move costs a reload and drops sessions); the lowest start breaks ties."""
    span = min(max_layers, num_layers)
    cands = {(s, s + span) for s in range(num_layers - span + 1)}
    cands.add(tuple(choose_range(num_layers, span, others)))
    here = swarm_score(num_layers, list(others) + [tuple(mine)])
    best = max(sorted(cands), key=lambda c: (swarm_score(num_layers, list(others) + [c]), -c[0]))
    if tuple(best) != tuple(mine) and swarm_score(num_layers, list(others) + [best]) > here:
        return best
    return None


def find_chain(entries: Sequence[dict], num_layers: int, start: int = 0) -> List[dict]:
    """Servers whose ranges chain exactly from layer ``start`` to ``num_layers`` (fewest hops;
    among equals the earliest-listed servers), or [] if the given servers do not cover it.
    (``start`` > 0: the replacement for one failed hop of a longer chain.)"""
    by_start: Dict[int, List[dict]] = {}
    for e in entries:
        by_start.setdefault(int(e["start"]), []).append(e)
    # breadth-first over layer boundaries: the first path that reaches num_layers has fewest hops
    prev: Dict[int, Tuple[int, dict]] = {}
    frontier = [start]
    seen = {start}
    while frontier:
        nxt = []
        for b in frontier:
            for e in by_start.get(b, []):
                end = int(e["end"])
                if end not in seen and end <= num_layers:
                    seen.add(end)
                    prev[end] = (b, e)
                    nxt.append(end)
        if num_layers in seen:
            break
        frontier = nxt
    if num_layers not in seen or num_layers == start:
        return []
    chain, b = [], num_layers
    while b != start:
        b0, e = prev[b]
        chain.append(e)
        b = b0
    return chain[::-1]


class Registry:
    """In-memory registry state (the service wraps it; tests use it directly)."""

    def __init__(self, claim_ttl: float = 900.0):
        self.claim_ttl = claim_ttl
        self._lock = threading.Lock()
        self._entries: Dict[str, dict] = {}   # url -> entry

    def _expire(self, now: float) -> None:
        for url in [u for u, e in self._entries.items() if e["expires"] < now]:
            del self._entries[url]

    def claim(self, model: str, num_layers: int, max_layers: int, url: str) -> Tuple[int, int]:
        with self._lock:
            now = time.monotonic()
            self._expire(now)
            self._entries.pop(url, None)   # a restarted server re-claims
            served = [(e["start"], e["end"]) for e in self._entries.values() if e["model"] == model]
            s, e = choose_range(num_layers, max_layers, served)
            self._entries[url] = {"url": url, "model": model, "start": s, "end": e,
                                  "num_layers": num_layers, "ready": False,
                                  "expires": now + self.claim_ttl}
            return s, e

    def announce(self, model: str, url: str, start: int, end: int, num_layers: int,
                 ttl: float) -> None:
        with self._lock:
            self._entries[url] = {"url": url, "model": model, "start": int(start),
                                  "end": int(end), "num_layers": int(num_layers), "ready": True,
                                  "expires": time.monotonic() + float(ttl)}

    def withdraw(self, url: str) -> None:
        with self._lock:
            self._entries.pop(url, None)

    def rebalance(self, model: str, url: str, num_layers: int,
                  max_layers: int) -> Optional[Tuple[int, int]]:
        """The range the ready server ``url`` should move to (recorded as its claim), or None."""
        with self._lock:
            now = time.monotonic()
            self._expire(now)
            me = self._entries.get(url)
            if me is None or not me["ready"] or me["model"] != model:
                return None
            others = [(e["start"], e["end"]) for u, e in self._entries.items()
                      if u != url and e["model"] == model]
            target = rebalance_target(num_layers, max_layers, others, (me["start"], me["end"]))
            if target is not None:
                self._entries[url] = {"url": url, "model": model, "start": target[0],
                                      "end": target[1], "num_layers": num_layers, "ready": False,
                                      "expires": now + self.claim_ttl}
            return target

    def servers(self, model: Optional[str] = None) -> List[dict]:
        with self._lock:
            self._expire(time.monotonic())
            return [{k: v for k, v in e.items() if k != "expires"}
                    for e in self._entries.values() if model is None or e["model"] == model]


def build_registry_app(reg: Optional[Registry] = None, token: Optional[str] = None):
    """The registry's HTTP service; ``token``: the shared secret the mutating endpoints require."""
    import hmac
    from fastapi import FastAPI, HTTPException
    reg = reg or Registry()
    app = FastAPI(title="distributed_llm_inference block registry")

    def _auth(request: Request) -> None:
        if token is None:
            return
        got = request.headers.get("authorization", "")
        if not hmac.compare_digest(got.encode(), f"Bearer {token}".encode()):
            raise HTTPException(401, "registry token required (Authorization: Bearer ...)")

    @app.post("/claim")
    async def claim(body: dict, request: Request):
        _auth(request)
        try:
            s, e = reg.claim(str(body["model"]), int(body["num_layers"]),
                             int(body["max_layers"]), str(body["url"]))
        except (KeyError, ValueError, TypeError) as ex:
            raise HTTPException(400, f"bad claim: {ex!r}")
        return {"start": s, "end": e}

    @app.post("/announce")
    async def announce(body: dict, request: Request):
        _auth(request)
        try:
            start, end, n = int(body["start"]), int(body["end"]), int(body["num_layers"])
            if not 0 <= start < end <= n:
                raise ValueError(f"range [{start}, {end}) outside [0, {n})")
            reg.announce(str(body["model"]), str(body["url"]), start, end, n,
                         float(body.get("ttl", 30.0)))
        except (KeyError, ValueError, TypeError) as ex:
            raise HTTPException(400, f"bad announce: {ex!r}")
        return {"ok": True}

    @app.post("/withdraw")
    async def withdraw(body: dict, request: Request):
        _auth(request)
        try:
            reg.withdraw(str(body["url"]))
        except (KeyError, TypeError) as ex:
            raise HTTPException(400, f"bad withdraw: {ex!r}")
        return {"ok": True}

    @app.post("/rebalance")
    async def rebalance(body: dict, request: Request):
        _auth(request)
        try:
            t = reg.rebalance(str(body["model"]), str(body["url"]), int(body["num_layers"]),
                              int(body["max_layers"]))
        except (KeyError, ValueError, TypeError) as ex:
            raise HTTPException(400, f"bad rebalance: {ex!r}")
        return {"move": t is not None, "start": t[0] if t else None, "end": t[1] if t else None}

    @app.get("/servers")
    async def servers(model: Optional[str] = None):
        return reg.servers(model)

    return app


def serve_registry(host: str = "127.0.0.1", port: int = 8099, token: Optional[str] = None) -> None:
    import uvicorn
    uvicorn.run(build_registry_app(token=token), host=host, port=port, log_level="warning")


class RegistryClient:
    def __init__(self, url: str, timeout: float = 30.0, token: Optional[str] = None):
        import requests
        self.url = url.rstrip("/")
        self.timeout = timeout
        self._s = requests.Session()
        self.token = token or None
        if token:
            self._s.headers["Authorization"] = f"Bearer {token}"

    def _post(self, path: str, body: dict) -> dict:
        r = self._s.post(self.url + path, json=body, timeout=self.timeout)
        if r.status_code != 200:
            raise RuntimeError(f"{self.url}{path}: HTTP {r.status_code}: {r.text[:300]}")
        return r.json()

    def claim(self, model: str, num_layers: int, max_layers: int, url: str) -> Tuple[int, int]:
        d = self._post("/claim", {"model": model, "num_layers": num_layers,
                                  "max_layers": max_layers, "url": url})
        return int(d["start"]), int(d["end"])

    def announce(self, model: str, url: str, start: int, end: int, num_layers: int,
                 ttl: float = 30.0) -> None:
        self._post("/announce", {"model": model, "url": url, "start": start, "end": end,
                                 "num_layers": num_layers, "ttl": ttl})

    def withdraw(self, url: str) -> None:
        self._post("/withdraw", {"url": url})

    def rebalance(self, model: str, url: str, num_layers: int,
                  max_layers: int) -> Optional[Tuple[int, int]]:
        d = self._post("/rebalance", {"model": model, "url": url, "num_layers": num_layers,
                                      "max_layers": max_layers})
        return (int(d["start"]), int(d["end"])) if d["move"] else None

    def servers(self, model: Optional[str] = None, ready_only: bool = True) -> List[dict]:
        r = self._s.get(self.url + "/servers", params={"model": model} if model else None,
                        timeout=self.timeout)
        r.raise_for_status()
        return [e for e in r.json() if e["ready"] or not ready_only]


def heartbeat_loop(client: RegistryClient, model: str, url: str, start: int, end: int,
                   num_layers: int, healthy, ttl: float = 30.0,
                   stop: Optional[threading.Event] = None,
                   current_range: Optional[Callable[[], Optional[Tuple[int, int]]]] = None
                   ) -> threading.Thread:
    """Background thread: announce this server while ``healthy()`` holds, every ttl / 3.
    ``current_range``: the range to announce, read at every beat (None: skip the beat -- the
    server is moving and its new claim must not be overwritten)."""
    stop = stop or threading.Event()

    def run():
        while not stop.is_set():
            try:
                rng = current_range() if current_range is not None else (start, end)
                if rng is not None and healthy():
                    client.announce(model, url, rng[0], rng[1], num_layers, ttl)
            except Exception:  # noqa: BLE001 - the registry may be restarting; keep trying
                pass
            stop.wait(ttl / 3)

    th = threading.Thread(target=run, name="registry-heartbeat", daemon=True)
    th.start()
    return th
