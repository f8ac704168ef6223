"""MI355X-native ForwardTacotron inference path."""
from . import jit as _jit  # noqa: F401  registers torch.ops.ftmi.* (TorchScript archives)
