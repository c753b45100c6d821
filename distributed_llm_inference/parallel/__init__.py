"""Pipeline parallelism across MI355X GPUs: RCCL P2P transport + driver/follower stage loops."""
from .transport import LoopbackTransport, RcclTransport, TorchDistTransport, Transport  # noqa: F401
