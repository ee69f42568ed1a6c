from .config import CfgNode, load_run_config, load_yaml, apply_overrides, RunConfig
from .misc import set_seed, setup_logging, print_model_size, model_size_bytes

__all__ = [
    "CfgNode", "load_run_config", "load_yaml", "apply_overrides", "RunConfig",
    "set_seed", "setup_logging", "print_model_size", "model_size_bytes",
]
