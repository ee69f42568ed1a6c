"""mingpt_distributed_amd: an MI355X-native (gfx950) minGPT training / inference framework.

Layers: ``ops`` (hand-written HIP kernels + autograd glue), ``models`` (GPT), ``optim`` (flat
buffers, fused AdamW), ``parallel`` (RCCL data parallel engine), ``trainer``, ``data``, ``bpe``,
``utils``.  See README.md and SURVEY.md.
"""
__version__ = "0.1.0"

from .models import GPT, GPTConfig, OptimizerConfig  # noqa: E402
from .optim import create_optimizer  # noqa: E402
from .trainer import GPTTrainer, GPTTrainerConfig, ModelSnapshot, Trainer  # noqa: E402
from .data import CharDataset, DataConfig  # noqa: E402
from .utils import CfgNode, set_seed, setup_logging, print_model_size  # noqa: E402

__all__ = ["GPT", "GPTConfig", "OptimizerConfig", "create_optimizer", "GPTTrainer", "GPTTrainerConfig",
           "ModelSnapshot", "Trainer", "CharDataset", "DataConfig", "CfgNode", "set_seed", "setup_logging",
           "print_model_size"]
