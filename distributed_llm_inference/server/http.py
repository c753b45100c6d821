"""HTTP front-end (FastAPI) for :class:`EngineService`.

Endpoints:
  POST /generate         {"prompt" | "prompt_ids", "max_tokens", "temperature", "top_k", "top_p",
                          "seed", "stop_token_ids", "ignore_eos", "stream"}
  POST /v1/completions   minimal OpenAI-compatible completion (non-streaming and SSE streaming)
  GET  /health           liveness + engine stats (503 when the engine loop died)
  GET  /metrics          Prometheus text format
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import Any, List, Optional

from ..runtime.sequence import SamplingParams
from .service import EngineService


def build_app(service: EngineService, tokenizer=None, model_name: str = "model",
              request_timeout_s: Optional[float] = None):
    """``request_timeout_s`` (or a request's ``timeout_s``): a request still running after that
    long is aborted (KV freed) and answered 504; a streaming client that disconnects aborts its
    sequence as well."""
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse

    app = FastAPI(title="distributed_llm_inference (MI355X)")

    def _encode(body: dict) -> List[int]:
        if body.get("prompt_ids") is not None:
            return [int(t) for t in body["prompt_ids"]]
        prompt = body.get("prompt")
        if prompt is None:
            raise HTTPException(400, "need 'prompt' or 'prompt_ids'")
        if isinstance(prompt, list):
            return [int(t) for t in prompt]
        if tokenizer is None:
            raise HTTPException(400, "no tokenizer loaded: send 'prompt_ids'")
        return tokenizer.encode(prompt)

    def _decode(ids: List[int]) -> Optional[str]:
        if tokenizer is None:
            return None
        return tokenizer.decode(ids, skip_special_tokens=True)

    def _params(body: dict) -> SamplingParams:
        try:
            return SamplingParams(
                max_tokens=int(body.get("max_tokens", 16)),
                temperature=float(body.get("temperature", 0.0)),
                top_k=int(body.get("top_k", 0) or 0), top_p=float(body.get("top_p", 1.0)),
                seed=body.get("seed"), stop_token_ids=body.get("stop_token_ids"),
                ignore_eos=bool(body.get("ignore_eos", False)))
        except ValueError as e:
            raise HTTPException(400, str(e))

    def _timeout(body: dict) -> Optional[float]:
        t = body.get("timeout_s", request_timeout_s)
        return float(t) if t is not None else None

    async def _result(fut, timeout: Optional[float]):
        try:
            return await asyncio.wait_for(asyncio.shield(asyncio.wrap_future(fut)), timeout)
        except asyncio.TimeoutError:
            service.abort(fut.seq_id)
            raise HTTPException(504, f"request timed out after {timeout} s (generation aborted)")

    async def _stream(q, fut=None, timeout: Optional[float] = None):
        """SSE token stream.  A client that disconnects (the generator is closed early) or a
        stream that outlives its timeout aborts the sequence, so its KV blocks are freed."""
        loop = asyncio.get_running_loop()
        deadline = time.monotonic() + timeout if timeout is not None else None
        finished = False
        try:
            while True:
                wait = None if deadline is None else max(0.0, deadline - time.monotonic())
                try:
                    tok = await asyncio.wait_for(loop.run_in_executor(None, q.get), wait)
                except asyncio.TimeoutError:
                    yield f"data: {json.dumps({'error': 'timeout'})}\n\n"
                    break
                if tok is None:
                    finished = True
                    break
                payload = {"token_id": tok}
                txt = _decode([tok])
                if txt is not None:
                    payload["text"] = txt
                yield f"data: {json.dumps(payload)}\n\n"
            if finished:
                yield "data: [DONE]\n\n"
        finally:
            if not finished and fut is not None:
                service.abort(fut.seq_id)

    @app.post("/generate")
    async def generate(body: dict):
        ids = _encode(body)
        params = _params(body)
        try:
            fut, q = service.submit(ids, params, stream=bool(body.get("stream")))
        except Exception as e:
            raise HTTPException(400, str(e))
        if q is not None:
            return StreamingResponse(_stream(q, fut=fut, timeout=_timeout(body)),
                                     media_type="text/event-stream")
        res = await _result(fut, _timeout(body))
        return {"output_ids": res.output_ids, "text": _decode(res.output_ids),
                "finish_reason": res.finish_reason,
                "usage": {"prompt_tokens": res.prompt_len,
                          "completion_tokens": len(res.output_ids)},
                "latency_s": round(res.latency_s, 4),
                "ttft_s": round(res.ttft_s, 4) if res.ttft_s is not None else None}

    @app.post("/v1/completions")
    async def completions(body: dict):
        ids = _encode(body)
        params = _params(body)
        fut, q = service.submit(ids, params, stream=bool(body.get("stream")))
        if q is not None:
            return StreamingResponse(_stream(q, fut=fut, timeout=_timeout(body)),
                                     media_type="text/event-stream")
        res = await _result(fut, _timeout(body))
        return {"id": f"cmpl-{res.seq_id}", "object": "text_completion", "created": int(time.time()),
                "model": model_name,
                "choices": [{"index": 0, "text": _decode(res.output_ids),
                             "token_ids": res.output_ids, "finish_reason": res.finish_reason}],
                "usage": {"prompt_tokens": res.prompt_len,
                          "completion_tokens": len(res.output_ids),
                          "total_tokens": res.prompt_len + len(res.output_ids)}}

    @app.get("/health")
    async def health():
        st = service.stats()
        return JSONResponse(st, status_code=200 if st["healthy"] else 503)

    @app.get("/metrics")
    async def metrics():
        st = service.stats()
        lines = []
        for k, v in st.items():
            if isinstance(v, bool):
                v = int(v)
            if isinstance(v, (int, float)):
                lines.append(f"dli_{k} {v}")
        for r, rec in enumerate(service.stage_stats()):   # per pipeline stage (rank)
            for k, v in (rec or {}).items():
                if isinstance(v, (int, float)):
                    lines.append(f'dli_stage_{k}{{stage="{r}"}} {v}')
        return PlainTextResponse("\n".join(lines) + "\n")

    return app


def serve(service: EngineService, host: str = "127.0.0.1", port: int = 8000, tokenizer=None,
          model_name: str = "model", request_timeout_s: Optional[float] = None) -> None:
    import uvicorn
    uvicorn.run(build_app(service, tokenizer, model_name, request_timeout_s), host=host, port=port,
                log_level="info")
