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
                                   "data"} -> msgpack {"shape", "dtype", "data"}
                                   (no block_id: every block of the worker, in order)
    POST /close_session            {"generation_id"}: free the session's KV on every block

Client: :class:`RemoteBlocks` (one server) and :class:`RemoteSequential` (a chain of servers
whose ranges tile [0, L) - the client side of the swarm: ``forward(gid, hidden)`` walks the
chain, ``close_session(gid)`` frees the session everywhere; ``from_registry`` finds the chain in
a block registry, server/registry.py, where ``block-serve --registry`` servers claim their layers).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import msgpack
import torch

try:   # module level: FastAPI resolves the (string) annotations of the handlers here
    from fastapi import Request
except ImportError:  # pragma: no cover - the client side needs no web framework
    Request = None

_DTYPES = {"bfloat16": torch.bfloat16, "float32": torch.float32, "float16": torch.float16}


def pack_tensor(t: torch.Tensor) -> dict:
    t = t.detach().contiguous().cpu()
    name = str(t.dtype).replace("torch.", "")
    if name not in _DTYPES:
        raise TypeError(f"unsupported dtype {t.dtype}")
    # raw bytes of the storage (bf16 has no numpy dtype: view as int16)
    raw = t.view(torch.int16) if t.dtype in (torch.bfloat16, torch.float16) else t
    return {"shape": list(t.shape), "dtype": name, "data": raw.numpy().tobytes()}


def unpack_tensor(d: dict) -> torch.Tensor:
    dt = _DTYPES[d["dtype"]]
    buf = bytearray(d["data"])
    if dt in (torch.bfloat16, torch.float16):
        return torch.frombuffer(buf, dtype=torch.int16).view(dt).reshape(d["shape"])
    return torch.frombuffer(buf, dtype=dt).reshape(d["shape"])


def build_block_app(worker):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import JSONResponse, Response

    app = FastAPI(title="distributed_llm_inference block server")

    @app.get("/info")
    async def info():
        return {"model": worker.spec.name, "start": worker.start, "end": worker.end,
                "hidden_size": worker.spec.hidden_size, "device": str(worker.device),
                "blocks": [dict(b) for b in worker.block_ids]}

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
        bid = body.get("block_id")
        if bid is not None and bid not in worker.blocks:
            raise HTTPException(404, f"unknown block {bid!r}")

        def run():
            y = worker.forward(bid, gid, x) if bid is not None else worker.forward_range(gid, x)
            return pack_tensor(y.to(x.dtype))

        out = await asyncio.get_running_loop().run_in_executor(None, run)
        return Response(msgpack.packb(out), media_type="application/msgpack")

    @app.post("/close_session")
    async def close_session(request: Request):
        body = await request.json()
        worker.close_session(body["generation_id"])
        return {"closed": body["generation_id"]}

    return app


def serve_blocks(worker, host: str = "127.0.0.1", port: int = 8100, registry=None,
                 url: Optional[str] = None, ttl: float = 30.0) -> None:
    """Serve ``worker`` over HTTP.  With ``registry`` (a :class:`RegistryClient`) the server is
    announced under ``url`` while its /health answers, and withdrawn when it stops."""
    import uvicorn
    worker.run()
    stop = None
    if registry is not None:
        import threading
        from .registry import heartbeat_loop
        url = url or f"http://{host}:{port}"
        probe = RemoteBlocks(url, timeout=5.0)
        stop = threading.Event()
        heartbeat_loop(registry, worker.spec.name, url, worker.start, worker.end,
                       worker.spec.num_layers, probe.healthy, ttl=ttl, stop=stop)
    try:
        uvicorn.run(build_block_app(worker), host=host, port=port, log_level="warning")
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
            r = self._s.get(self.url + "/info", timeout=self.timeout)
            r.raise_for_status()
            self._info = r.json()
        return self._info

    def healthy(self) -> bool:
        try:
            return self._s.get(self.url + "/health", timeout=5).status_code == 200
        except Exception:  # noqa: BLE001
            return False

    def forward(self, generation_id: str, hidden: torch.Tensor,
                block_id: Optional[str] = None) -> torch.Tensor:
        body = pack_tensor(hidden)
        body["generation_id"] = generation_id
        if block_id is not None:
            body["block_id"] = block_id
        r = self._s.post(self.url + "/forward", data=msgpack.packb(body),
                         headers={"Content-Type": "application/msgpack"}, timeout=self.timeout)
        if r.status_code != 200:
            raise RuntimeError(f"{self.url}/forward: HTTP {r.status_code}: {r.text[:500]}")
        return unpack_tensor(msgpack.unpackb(r.content))

    def close_session(self, generation_id: str) -> None:
        r = self._s.post(self.url + "/close_session", json={"generation_id": generation_id},
                         timeout=self.timeout)
        r.raise_for_status()


class RemoteSequential:
    """A chain of block servers covering consecutive layer ranges (the swarm's client side)."""

    def __init__(self, urls: Sequence[str], timeout: float = 120.0):
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

    @classmethod
    def from_registry(cls, registry_url: str, model: str, timeout: float = 120.0,
                      wait_s: float = 0.0) -> "RemoteSequential":
        """The chain of ready servers listed by a block registry (server/registry.py) that
        covers ``model`` from layer 0 to its last layer; ``wait_s``: keep polling that long
        for the swarm to cover it."""
        import time
        from ..config import resolve_model
        from .registry import RegistryClient, find_chain
        reg = RegistryClient(registry_url)
        try:
            name = resolve_model(model).name
        except ValueError:
            name = model
        deadline = time.monotonic() + wait_s
        while True:
            entries = reg.servers(name)
            L = max([int(e["num_layers"]) for e in entries] + [0])
            chain = find_chain(entries, L) if L else []
            if chain or time.monotonic() >= deadline:
                break
            time.sleep(0.5)
        if not chain:
            raise LookupError(f"registry {registry_url} lists no chain of ready servers covering "
                              f"{name} (servers: {[(e['start'], e['end']) for e in entries]})")
        return cls([e["url"] for e in chain], timeout=timeout)

    def forward(self, generation_id: str, hidden: torch.Tensor) -> torch.Tensor:
        for s in self.servers:
            hidden = s.forward(generation_id, hidden)
        return hidden

    __call__ = forward

    def close_session(self, generation_id: str) -> None:
        for s in self.servers:
            s.close_session(generation_id)
