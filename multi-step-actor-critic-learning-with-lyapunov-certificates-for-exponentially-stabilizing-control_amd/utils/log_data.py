"""Running averages of logged scalars (same contract as RL/utils/log_data.py:5-35)."""
from typing import Sequence, Union


class LogData:
    def __init__(self):
        self.data = {}
        self.counter = {}

    def _one(self, d: dict):
        for k, v in d.items():
            c = self.counter.get(k, 0)
            self.data[k] = v if c == 0 else (self.data[k] * c + v) / (c + 1)
            self.counter[k] = c + 1

    def add_average(self, d: Union[dict, Sequence[dict]]):
        if isinstance(d, dict):
            self._one(d)
        elif isinstance(d, Sequence):
            for item in d:
                self._one(item)
        else:
            raise TypeError(f"Unsupported type {type(d)} for add_average!")

    def pop(self) -> dict:
        out, self.data, self.counter = dict(self.data), {}, {}
        return out
