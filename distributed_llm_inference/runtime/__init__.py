"""Runtime: sequences, scheduler, stage executor (hipGraph decode), engine construction."""
from .executor import StageExecutor, StepPlan  # noqa: F401
from .scheduler import Scheduler  # noqa: F401
from .sequence import SamplingParams, Sequence, SeqStatus  # noqa: F401

_ENGINE = ("EngineConfig", "LLMEngine", "build_executor", "init_pipeline_rank")


def __getattr__(name):
    # engine.py imports parallel.pipeline, which imports this package's executor: resolving the
    # engine names lazily lets either package be imported first (no import cycle)
    if name in _ENGINE:
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
