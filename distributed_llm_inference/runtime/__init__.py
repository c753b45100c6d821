"""Runtime: sequences, scheduler, stage executor (hipGraph decode), engine construction."""
from .executor import StageExecutor, StepPlan  # noqa: F401
from .scheduler import Scheduler  # noqa: F401
from .sequence import SamplingParams, Sequence, SeqStatus  # noqa: F401
from .engine import EngineConfig, LLMEngine, build_executor, init_pipeline_rank  # noqa: F401
