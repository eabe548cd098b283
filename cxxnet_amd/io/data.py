"""DataBatch and the iterator interface (reference src/io/data.h:18-186)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch


@dataclass
class DataBatch:
    """One mini-batch: data (b,c,h,w) float32, label (b, label_width) float32,
    inst_index (b,) uint32, num_batch_padd = padded tail rows, extra_data list."""
    data: torch.Tensor
    label: torch.Tensor
    inst_index: Optional[np.ndarray] = None
    num_batch_padd: int = 0
    extra_data: List[torch.Tensor] = field(default_factory=list)

    @property
    def batch_size(self):
        return int(self.data.shape[0])


class DataIterator:
    """IIterator<DataBatch>: set_param -> init -> (before_first, next/value)*."""

    def set_param(self, name: str, val: str):
        pass

    def init(self):
        pass

    def before_first(self):
        raise NotImplementedError

    def next(self) -> bool:
        raise NotImplementedError

    def value(self) -> DataBatch:
        raise NotImplementedError

    def __iter__(self):
        self.before_first()
        while self.next():
            yield self.value()

    def close(self):
        pass
