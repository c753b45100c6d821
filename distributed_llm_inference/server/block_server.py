"""Remote hidden-state block forward: a worker's layer range served to other processes.

The reference is the server side of a Petals-style swarm: a client holds the embedding and the
head, and sends ``hidden_states`` + ``generation_id`` to the block server that owns layers
[a, b) (reference server/backend.py:31-42 - the hivemind TaskPool fed by ``ConnectionHandler``
RPCs; server/worker.py:9-20 - one backend per block of the worker's range).  hivemind's libp2p /
protobuf wire is replaced by plain HTTP with a msgpack body (header + raw tensor bytes, no
pickling), and the server side is this framework's :class:`InferenceWorker`, whose batching
pool packs the concurrent sessions' steps into one varlen forward on the paged-KV kernels.

Server (``distribute block-serve --model M --start a --end b --port P``)::

    GET  /info                     {"model", "start", "end", "hidden_size", "blocks": [...]}
    GET  /health                   200 while every block's pool is alive
    POST /forward                  msgpack {"generation_id", "block_id"?, "shape", "dtype",
                                   "data", "attention_mask"?, "position_ids"?,
                                   "output_hidden_states"?} -> msgpack {"shape", "dtype", "data",
                                   "hidden_states"?: [tensor, ...]}
                                   (no block_id: every block of the worker, in order; the optional
                                   fields are the reference stage API's arguments, reference
                                   models/llama/model.py:25-33, tensors packed like the hidden)
    POST /close_session            {"generation_id"}: free the session's KV on every block

Client: :class:`RemoteBlocks` (one server) and :class:`RemoteSequential` (a chain of servers
whose ranges tile [0, L) - the client side of the swarm: ``forward(gid, hidden, ...)`` walks the
chain, ``close_session(gid)`` frees the session everywhere; ``from_registry`` finds the chain in
a block registry, server/registry.py, where ``block-serve --registry`` servers claim their layers).

Failover (reference server/server.py:15-23: the swarm survives unhealthy servers): the client
keeps, per session, the inputs it sent to every layer range.  When a hop fails (connection error,
timeout or HTTP 5xx) it re-resolves that range from the registry (any ready servers chaining it,
the dead one excluded), replays the session's history into them to rebuild their KV, and carries
on - the outputs equal an uninterrupted run.  A session that cannot be recovered is closed on
every surviving server before the error is raised, so no KV is orphaned.
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List, Optional, Sequence, Tuple

import msgpack
import torch

try:   # module level: FastAPI resolves the (string) annotations of the handlers here
    from fastapi import Request
except ImportError:  # pragma: no cover - the client side needs no web framework
    Request = None

log = logging.getLogger(__name__)

_DTYPES = {"bfloat16": torch.bfloat16, "float32": torch.float32, "float16": torch.float16,
           "int64": torch.int64, "int32": torch.int32, "bool": torch.bool}
_STAGE_KWARGS = ("attention_mask", "position_ids")


def pack_tensor(t: torch.Tensor) -> dict:
    t = t.detach().contiguous().cpu()
    name = str(t.dtype).replace("torch.", "")
    if name not in _DTYPES:
        raise TypeError(f"unsupported dtype {t.dtype}")
    # raw bytes of the storage (bf16 has no numpy dtype: view as int16; bool as uint8)
    raw = (t.view(torch.int16) if t.dtype in (torch.bfloat16, torch.float16)
           else t.view(torch.uint8) if t.dtype == torch.bool else t)
    return {"shape": list(t.shape), "dtype": name, "data": raw.numpy().tobytes()}


def unpack_tensor(d: dict) -> torch.Tensor:
    dt = _DTYPES[d["dtype"]]
    buf = bytearray(d["data"])
    if dt in (torch.bfloat16, torch.float16):
        return torch.frombuffer(buf, dtype=torch.int16).view(dt).reshape(d["shape"])
    if dt == torch.bool:
        return torch.frombuffer(buf, dtype=torch.uint8).view(torch.bool).reshape(d["shape"])
    return torch.frombuffer(buf, dtype=dt).reshape(d["shape"])


class HopFailure(RuntimeError):
    """A block server could not be reached or failed on its side (connection error, timeout,
    HTTP 5xx): the hop is replaceable.  Client errors (4xx) are plain RuntimeErrors."""


class HopMoved(HopFailure):
    """The server now serves other layers (swarm rebalancing): re-resolve its old range."""


def build_block_app(worker, rebalance=None, token=None):
    """The block server's HTTP service; ``rebalance``: a callable running one rebalancing round
    (:func:`rebalance_once`) behind POST /rebalance, for operators and tests.  ``token``: the
    registry's shared token (``--registry-token``), then required by POST /rebalance as well
    (``Authorization: Bearer ...``), since a move changes what the swarm serves; without a
    token only loopback clients may ask for a move."""
    import hmac
    from fastapi import FastAPI, HTTPException, Request
    from fastapi.responses import JSONResponse, Response

    app = FastAPI(title="distributed_llm_inference block server")

    @app.post("/rebalance")
    async def rebalance_now(request: Request):
        import asyncio
        if token is not None and not hmac.compare_digest(
                request.headers.get("authorization", "").encode(), f"Bearer {token}".encode()):
            raise HTTPException(401, "registry token required (Authorization: Bearer ...)")
        if token is None and (request.client is None or
                              request.client.host not in ("127.0.0.1", "::1", "localhost")):
            # no shared secret configured: a move reloads weights on this GPU host, so only
            # the host itself may ask for one
            raise HTTPException(403, "POST /rebalance without a registry token: loopback only")
        if rebalance is None:
            raise HTTPException(404, "this server has no registry to rebalance against")
        moved = await asyncio.get_running_loop().run_in_executor(None, rebalance)
        return {"moved": moved is not None, "start": worker.start, "end": worker.end}

    @app.get("/info")
    async def info():
        return {"model": worker.spec.name, "start": worker.start, "end": worker.end,
                "hidden_size": worker.spec.hidden_size, "device": str(worker.device),
                "blocks": [dict(b) for b in worker.block_ids], "sessions": worker.sessions()}

    @app.get("/health")
    async def health():
        ok = worker.is_healthy()
        return JSONResponse({"healthy": ok}, status_code=200 if ok else 503)

    @app.post("/forward")
    async def forward(request: Request):
        import asyncio
        body = msgpack.unpackb(await request.body())
        gid = body.get("generation_id")
        if not gid:
            raise HTTPException(400, "generation_id is required")
        x = unpack_tensor(body)
        if x.dim() != 3 or x.shape[-1] != worker.spec.hidden_size:
            raise HTTPException(400, f"hidden must be [B, T, {worker.spec.hidden_size}], "
                                     f"got {list(x.shape)}")
        want = body.get("expect_range")
        if want is not None and (int(want[0]), int(want[1])) != (worker.start, worker.end):
            # the client's chain predates a move of this server (rebalancing): 409, it re-resolves
            raise HTTPException(409, f"moved: serving [{worker.start}, {worker.end}), "
                                     f"not [{want[0]}, {want[1]})")
        bid = body.get("block_id")
        if bid is not None and bid not in worker.blocks:
            raise HTTPException(404, f"unknown block {bid!r}")
        kw = {k: unpack_tensor(body[k]) for k in _STAGE_KWARGS if body.get(k) is not None}
        if body.get("output_hidden_states"):
            kw["output_hidden_states"] = True

        def run():
            y = worker.forward(bid, gid, x, **kw) if bid is not None else \
                worker.forward_range(gid, x, **kw)
            if kw.get("output_hidden_states"):
                y, hs = y
                out = pack_tensor(y.to(x.dtype))
                out["hidden_states"] = [pack_tensor(h.to(x.dtype)) for h in hs]
                return out
            return pack_tensor(y.to(x.dtype))

        from .worker import WorkerMoving
        try:
            out = await asyncio.get_running_loop().run_in_executor(None, run)
        except WorkerMoving as e:   # loading another range: re-resolve (not a dead server)
            raise HTTPException(409, f"moving: {e}")
        except (ValueError, MemoryError) as e:   # a bad request / no KV room: the client's call
            raise HTTPException(422, f"{type(e).__name__}: {e}")
        except KeyError as e:   # the worker moved while this request walked its blocks
            raise HTTPException(409, f"moved: {e!r}")
        return Response(msgpack.packb(out), media_type="application/msgpack")

    @app.post("/close_session")
    async def close_session(request: Request):
        body = await request.json()
        worker.close_session(body["generation_id"])
        return {"closed": body["generation_id"]}

    return app


def rebalance_once(worker, registry, url: str, max_layers: int, moving) -> Optional[Tuple[int, int]]:
    """One rebalancing round: if the worker holds no sessions and the registry says moving to
    less-served layers helps the swarm (registry.rebalance_target, recorded there as this
    server's claim), load them, swap them in (InferenceWorker.move_to) and announce the new
    range.  ``moving`` pauses the heartbeat meanwhile, so it never re-announces the old range
    over the new claim.  Returns the new range, or None."""
    if worker.sessions():
        return None   # a move would drop their KV: wait until the server is idle
    target = registry.rebalance(worker.spec.name, url, worker.spec.num_layers, max_layers)
    if target is None:
        return None
    moving.set()
    try:
        old = (worker.start, worker.end)
        try:
            # re-checked under the worker's swap lock: a session opened since the check above
            # (or during the load, which refuses new sessions) abandons the move
            worker.move_to(*target, require_idle=True)
        except Exception:   # noqa: BLE001 - e.g. no memory for the new layers: stay
            log.exception("move [%d, %d) -> %s failed; staying", old[0], old[1], target)
        registry.announce(worker.spec.name, url, worker.start, worker.end,
                          worker.spec.num_layers)
        log.warning("rebalanced: layers [%d, %d) -> [%d, %d)", old[0], old[1], worker.start,
                    worker.end)
        return (worker.start, worker.end) if (worker.start, worker.end) != old else None
    finally:
        moving.clear()


def rebalance_loop(worker, registry, url: str, max_layers: int, period_s: float,
                   stop, moving) -> "threading.Thread":
    """:func:`rebalance_once` every ``period_s`` until ``stop``."""
    import threading

    def run():
        while not stop.wait(period_s):
            try:
                rebalance_once(worker, registry, url, max_layers, moving)
            except Exception:   # noqa: BLE001 - the registry may be restarting; keep trying
                log.debug("rebalance round failed", exc_info=True)

    th = threading.Thread(target=run, name="block-rebalance", daemon=True)
    th.start()
    return th


def serve_blocks(worker, host: str = "127.0.0.1", port: int = 8100, registry=None,
                 url: Optional[str] = None, ttl: float = 30.0, rebalance_s: float = 0.0,
                 max_layers: Optional[int] = None) -> None:
    """Serve ``worker`` over HTTP.  With ``registry`` (a :class:`RegistryClient`) the server is
    announced under ``url`` while its /health answers, and withdrawn when it stops;
    ``rebalance_s`` > 0: every that many seconds it may move to less-served layers
    (:func:`rebalance_loop`, at most ``max_layers`` of them)."""
    import uvicorn
    worker.run()
    stop = None
    if registry is not None:
        import threading
        from .registry import heartbeat_loop
        url = url or f"http://{host}:{port}"
        probe = RemoteBlocks(url, timeout=5.0)
        stop = threading.Event()
        moving = threading.Event()
        heartbeat_loop(registry, worker.spec.name, url, worker.start, worker.end,
                       worker.spec.num_layers, probe.healthy, ttl=ttl, stop=stop,
                       current_range=lambda: None if moving.is_set() else (worker.start,
                                                                             worker.end))
        span = max_layers or (worker.end - worker.start)
        rebalance = lambda: rebalance_once(worker, registry, url, span, moving)  # noqa: E731
        if rebalance_s > 0:
            rebalance_loop(worker, registry, url, span, rebalance_s, stop, moving)
    try:
        uvicorn.run(build_block_app(worker, rebalance if registry is not None else None,
                                    token=getattr(registry, "token", None)),
                    host=host, port=port, log_level="warning")
    finally:
        if registry is not None:
            stop.set()
            try:
                registry.withdraw(url)
            except Exception:  # noqa: BLE001 - best effort: the entry also expires after ttl
                pass


class RemoteBlocks:
    """Client of one block server."""

    def __init__(self, url: str, timeout: float = 120.0):
        import requests
        self.url = url.rstrip("/")
        self.timeout = timeout
        self._s = requests.Session()
        self._info: Optional[dict] = None

    def info(self) -> dict:
        if self._info is None:
            import requests
            try:
                r = self._s.get(self.url + "/info", timeout=self.timeout)
            except requests.RequestException as e:
                raise HopFailure(f"{self.url}/info: {e!r}") from e
            if r.status_code >= 500:
                raise HopFailure(f"{self.url}/info: HTTP {r.status_code}")
            r.raise_for_status()
            self._info = r.json()
        return self._info

    def sessions(self) -> List[str]:
        """The generation ids currently holding KV on the server (fresh, not cached)."""
        r = self._s.get(self.url + "/info", timeout=self.timeout)
        r.raise_for_status()
        return list(r.json().get("sessions", []))

    @property
    def range(self) -> Tuple[int, int]:
        i = self.info()
        return int(i["start"]), int(i["end"])

    def healthy(self) -> bool:
        try:
            return self._s.get(self.url + "/health", timeout=5).status_code == 200
        except Exception:  # noqa: BLE001
            return False

    def forward(self, generation_id: str, hidden: torch.Tensor, block_id: Optional[str] = None,
                attention_mask: Optional[torch.Tensor] = None,
                position_ids: Optional[torch.Tensor] = None,
                output_hidden_states: bool = False):
        """The server's layers on ``hidden [B, T, H]``; returns the hidden states, or
        ``(hidden, all_hidden_states)`` with ``output_hidden_states``.  Raises
        :class:`HopFailure` when the server is unreachable or fails on its side."""
        import requests
        body = pack_tensor(hidden)
        body["generation_id"] = generation_id
        if block_id is not None:
            body["block_id"] = block_id
        if attention_mask is not None:
            body["attention_mask"] = pack_tensor(attention_mask)
        if position_ids is not None:
            body["position_ids"] = pack_tensor(position_ids)
        if output_hidden_states:
            body["output_hidden_states"] = True
        body["expect_range"] = list(self.range)   # a moved server answers 409
        try:
            r = self._s.post(self.url + "/forward", data=msgpack.packb(body),
                             headers={"Content-Type": "application/msgpack"},
                             timeout=self.timeout)
        except requests.RequestException as e:
            raise HopFailure(f"{self.url}/forward: {e!r}") from e
        if r.status_code >= 500:
            raise HopFailure(f"{self.url}/forward: HTTP {r.status_code}: {r.text[:300]}")
        if r.status_code == 409:
            raise HopMoved(f"{self.url}/forward: {r.text[:300]}")
        if r.status_code != 200:
            raise RuntimeError(f"{self.url}/forward: HTTP {r.status_code}: {r.text[:500]}")
        d = msgpack.unpackb(r.content)
        y = unpack_tensor(d)
        if output_hidden_states:
            return y, tuple(unpack_tensor(h) for h in d.get("hidden_states", []))
        return y

    def close_session(self, generation_id: str) -> None:
        r = self._s.post(self.url + "/close_session", json={"generation_id": generation_id},
                         timeout=self.timeout)
        r.raise_for_status()


class ReplayFailure(HopFailure):
    """A replacement server failed while a session's history was replayed into it."""

    def __init__(self, msg: str, url: str):
        super().__init__(msg)
        self.url = url


def _concat_history(inputs: List[tuple]) -> Optional[tuple]:
    """One chunk equivalent to a session's recorded steps into a layer range: the hidden inputs
    concatenated along T, the 2-D padding masks along T (ones where a step had none), and the
    RoPE positions every step used - its explicit ``position_ids``, else the server's default
    (tokens cached so far + arange over the step's real tokens).  Replayed as ONE chunked
    prefill, this writes the same KV as the steps did one by one (causal attention over the
    same keys).  None when a step carried a 4-D mask (no single-chunk equivalent)."""
    hs, ams, poss = [], [], []
    seen = None   # per row: real tokens cached so far
    for h, kw in inputs:
        B, T = h.shape[0], h.shape[1]
        am = kw.get("attention_mask")
        if am is not None and am.dim() != 2:
            return None
        am = torch.ones(B, T, dtype=torch.bool) if am is None else am[:, -T:].to(torch.bool)
        if seen is None:
            seen = torch.zeros(B, dtype=torch.long)
        pid = kw.get("position_ids")
        if pid is not None:
            pos = pid[:, -T:].to(torch.long).expand(B, -1)
        else:
            pos = seen[:, None] + torch.cumsum(am.to(torch.long), 1) - 1
        seen = seen + am.sum(1)
        hs.append(h)
        ams.append(am)
        poss.append(pos)
    kw = {"position_ids": torch.cat(poss, 1)}
    am = torch.cat(ams, 1)
    if not bool(am.all()):
        kw["attention_mask"] = am.to(torch.long)
    return torch.cat(hs, 1), kw


class RemoteSequential:
    """A chain of block servers covering consecutive layer ranges (the swarm's client side).

    With a ``registry`` (``from_registry``) a failed hop is replaced by ready servers from the
    registry and the session's history is replayed into them (module docstring); without one a
    failure closes the session on the surviving servers and raises.

    History and its memory bound: per open session the client keeps the inputs it sent to each
    layer range (hidden ``[B, T, H]`` + the stage kwargs of every step) - ``T_total x H x 2``
    bytes per range in bf16, e.g. 16 KB per token per range for a 70B model.  A session whose
    recorded tokens exceed ``max_history_tokens`` drops its history and can no longer be
    recovered: if its range fails it is closed on every surviving server and a later forward on
    it raises (``lost``).  ``close_session`` frees the history.  On failover every session's
    history for the failed range is replayed as ONE concatenated chunk per replacement server
    (a chunked prefill; one call per server and session, whatever the number of steps)."""

    def __init__(self, urls: Sequence[str], timeout: float = 120.0, registry=None,
                 model: Optional[str] = None, failover_wait_s: float = 30.0,
                 max_failovers: int = 4, max_history_tokens: int = 32768):
        self.timeout = timeout
        self.servers: List[RemoteBlocks] = [RemoteBlocks(u, timeout) for u in urls]
        infos = [s.info() for s in self.servers]
        order = sorted(range(len(infos)), key=lambda i: infos[i]["start"])
        self.servers = [self.servers[i] for i in order]
        infos = [infos[i] for i in order]
        for a, b in zip(infos, infos[1:]):
            if a["end"] != b["start"]:
                raise ValueError(f"layer ranges do not chain: [{a['start']},{a['end']}) then "
                                 f"[{b['start']},{b['end']})")
        self.start, self.end = infos[0]["start"], infos[-1]["end"]
        self.registry, self.model = registry, model or infos[0]["model"]
        self.failover_wait_s, self.max_failovers = failover_wait_s, max_failovers
        self.max_history_tokens = max_history_tokens
        # per session: the inputs sent to each layer range, in order (hidden, kwargs)
        self._history: Dict[str, Dict[Tuple[int, int], List[tuple]]] = {}
        self._hist_tokens: Dict[str, int] = {}
        self.unrecoverable: set = set()   # sessions past max_history_tokens (no history kept)
        self.lost: set = set()            # sessions closed by a failover they could not survive
        self.dead: set = set()
        self.failovers = 0
        self.replay_calls = 0             # /forward calls made by replays (tests, metrics)

    @classmethod
    def from_registry(cls, registry_url: str, model: str, timeout: float = 120.0,
                      wait_s: float = 0.0, token: Optional[str] = None,
                      failover_wait_s: float = 30.0, **kw) -> "RemoteSequential":
        """The chain of ready servers listed by a block registry (server/registry.py) that
        covers ``model`` from layer 0 to its last layer; ``wait_s``: keep polling that long
        for the swarm to cover it.  The registry also serves failed hops' replacements."""
        from ..config import resolve_model
        from .registry import RegistryClient, find_chain
        reg = RegistryClient(registry_url, token=token)
        try:
            name = resolve_model(model).name
        except ValueError:
            name = model
        deadline = time.monotonic() + wait_s
        gone: set = set()   # listed until their ttl lapses, but not answering
        while True:
            entries = [e for e in reg.servers(name) if e["url"] not in gone]
            L = max([int(e["num_layers"]) for e in entries] + [0])
            chain = find_chain(entries, L) if L else []
            dead = [e["url"] for e in chain if not RemoteBlocks(e["url"], 5.0).healthy()]
            if dead:
                gone.update(dead)
                continue
            if chain or time.monotonic() >= deadline:
                break
            time.sleep(0.5)
        if not chain:
            raise LookupError(f"registry {registry_url} lists no chain of ready servers covering "
                              f"{name} (servers: {[(e['start'], e['end']) for e in entries]})")
        return cls([e["url"] for e in chain], timeout=timeout, registry=reg, model=name,
                   failover_wait_s=failover_wait_s, **kw)

    # ------------------------------------------------------------------ forward
    def forward(self, generation_id: str, hidden: torch.Tensor,
                attention_mask: Optional[torch.Tensor] = None,
                position_ids: Optional[torch.Tensor] = None,
                output_hidden_states: bool = False):
        """Walk the chain (the reference stage API over the whole model range).  Returns the
        hidden states, or ``(hidden, all_hidden_states)`` with ``output_hidden_states``."""
        if generation_id in self.lost:
            raise RuntimeError(f"session {generation_id!r} was lost in a failover (its history "
                               f"exceeded max_history_tokens={self.max_history_tokens})")
        kw = {}
        if attention_mask is not None:
            kw["attention_mask"] = attention_mask
        if position_ids is not None:
            kw["position_ids"] = position_ids
        keep = generation_id not in self.unrecoverable
        if keep:
            n = self._hist_tokens.get(generation_id, 0) + int(hidden.shape[1])
            if n > self.max_history_tokens:
                keep = False
                self.unrecoverable.add(generation_id)
                self._history.pop(generation_id, None)
                self._hist_tokens.pop(generation_id, None)
                log.warning("session %r: history past %d tokens dropped; it can no longer be "
                            "recovered from a server failure", generation_id,
                            self.max_history_tokens)
            else:
                self._hist_tokens[generation_id] = n
        hist = self._history.setdefault(generation_id, {}) if keep else None
        hs: list = []
        i = 0
        while i < len(self.servers):
            s = self.servers[i]
            try:
                out = s.forward(generation_id, hidden, output_hidden_states=output_hidden_states,
                                **kw)
            except HopFailure as e:
                self._failover(i, generation_id, e)
                if generation_id in self.lost:
                    raise RuntimeError(f"session {generation_id!r} was lost in the failover of "
                                       f"{e}") from e
                continue   # the replacement chain now sits at position i
            if hist is not None:
                hist.setdefault(s.range, []).append((hidden, kw))
            if output_hidden_states:
                out, h = out
                hs = hs[:-1] + list(h)
            hidden = out
            i += 1
        return (hidden, tuple(hs)) if output_hidden_states else hidden

    __call__ = forward

    def _failover(self, i: int, generation_id: str, err: Exception) -> None:
        """Replace hop ``i`` (its layer range) with ready servers from the registry and replay
        the history of EVERY open session into them (their KV for this range was on the dead
        server).  Every replacement whose replay fails is excluded; attempts are bounded by
        ``max_failovers`` and ``failover_wait_s``.  Raises - after closing the sessions on the
        surviving servers - when no replacement can be found."""
        failed = self.servers[i]
        a, b = failed.range
        if not isinstance(err, HopMoved):   # a moved server is alive, just elsewhere now
            self.dead.add(failed.url)
        log.warning("block server %s (layers [%d, %d)) failed: %s; re-resolving", failed.url, a,
                    b, err)
        last_err: Exception = err
        deadline = time.monotonic() + self.failover_wait_s
        attempts = 0
        while (self.registry is not None and self.failovers < self.max_failovers
               and attempts < self.max_failovers and time.monotonic() <= deadline):
            repl = self._resolve(a, b)
            if repl is None:
                time.sleep(0.5)
                continue
            attempts += 1
            try:
                self._replay(repl, (a, b))
            except HopFailure as e2:
                # the server that failed the replay is out whatever its /health says (a
                # persistent 5xx on /forward, a timeout, or a move behind a 409)
                self.dead.add(getattr(e2, "url", None) or repl[0].url)
                last_err = e2
                time.sleep(0.5)
                continue
            self.servers[i:i + 1] = repl
            self.failovers += 1
            log.warning("layers [%d, %d) now served by %s", a, b, [s.url for s in repl])
            return
        self._abandon(exclude={failed.url})
        raise RuntimeError(f"block server {failed.url} (layers [{a}, {b})) failed and no "
                           f"replacement was found: {last_err}") from last_err

    def _resolve(self, a: int, b: int) -> Optional[List[RemoteBlocks]]:
        from .registry import find_chain
        try:
            entries = [e for e in self.registry.servers(self.model) if e["url"] not in self.dead]
        except Exception:  # noqa: BLE001 - registry unreachable right now: retry until deadline
            return None
        chain = find_chain(entries, b, start=a)
        if not chain:
            return None
        repl = [RemoteBlocks(e["url"], self.timeout) for e in chain]
        for s in repl:
            if not s.healthy():   # listed until its ttl lapses, but already gone
                self.dead.add(s.url)
                return None
        return repl

    def _replay(self, repl: List[RemoteBlocks], rng: Tuple[int, int]) -> None:
        """Rebuild every open session's KV for layer range ``rng`` on the replacement servers:
        each server, in order, gets the session's recorded inputs for the range as ONE chunk
        (:func:`_concat_history`; per step only for 4-D masks) - the outputs of server k are the
        inputs of server k+1.  Atomic: the new ranges' history is committed only when every
        session has replayed; on a failure the sessions already replayed are closed on the
        replacements (no duplicated KV on a retry) and :class:`ReplayFailure` names the server.
        Sessions that kept no history (``unrecoverable``) are closed everywhere and ``lost``."""
        new_hist: Dict[str, Dict[Tuple[int, int], List[tuple]]] = {}
        done: List[str] = []
        try:
            for gid, hist in self._history.items():
                inputs = hist.get(rng, [])
                if not inputs:
                    continue
                per = {}
                cat = _concat_history(inputs)
                for s in repl:
                    steps = [cat] if cat is not None else inputs
                    per[s.range] = [cat] if cat is not None else list(inputs)
                    outs = []
                    for h, kw in steps:
                        try:
                            y = s.forward(gid, h, **kw)
                        except HopFailure as e:
                            raise ReplayFailure(f"replay of {gid!r} into {s.url}: {e}", s.url) from e
                        self.replay_calls += 1
                        outs.append((y, kw))
                    if cat is not None:
                        cat = outs[0]
                    else:
                        inputs = outs
                done.append(gid)
                new_hist[gid] = per
        except HopFailure:
            for gid in done:
                for s in repl:
                    try:
                        s.close_session(gid)
                    except Exception:  # noqa: BLE001 - best effort: it may be the failed one
                        pass
            raise
        for gid, per in new_hist.items():
            hist = self._history[gid]
            hist.pop(rng, None)
            hist.update(per)
        for gid in list(self.unrecoverable):
            if gid in self.lost:
                continue
            self.lost.add(gid)
            for s in self.servers:
                if s.url in self.dead:
                    continue
                try:
                    s.close_session(gid)
                except Exception:  # noqa: BLE001
                    pass

    def _abandon(self, exclude=()) -> None:
        """Close every session on the servers still alive (no orphaned KV)."""
        for gid in set(self._history) | self.unrecoverable:
            for s in self.servers:
                if s.url in exclude or s.url in self.dead:
                    continue
                try:
                    s.close_session(gid)
                except Exception:  # noqa: BLE001 - best effort: the server may be gone too
                    pass
        self._history.clear()
        self._hist_tokens.clear()

    def close_session(self, generation_id: str) -> None:
        self._history.pop(generation_id, None)
        self._hist_tokens.pop(generation_id, None)
        self.unrecoverable.discard(generation_id)
        if generation_id in self.lost:
            self.lost.discard(generation_id)
            return
        for s in self.servers:
            s.close_session(generation_id)
