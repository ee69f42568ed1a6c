from .char_dataset import CharDataset, DataConfig
from .datasets import AdditionDataset, SortDataset, SyntheticTokens

__all__ = ["CharDataset", "DataConfig", "AdditionDataset", "SortDataset", "SyntheticTokens"]
