"""``dplasma_info_t``: string key/value options attached to a call.

Same operations as the reference (``src/utils/dplasma_info.c:43-152``):
create / set / get / get_nkeys / get_nthkey / delete / free.  Keys such as
``DPLASMA:GEMM:GPU:look_ahead`` tune individual algorithms
(``src/zgemm_wrapper.c:251-333``).
"""
from __future__ import annotations

from typing import Optional


class Info:
    MAX_KEY = 255
    MAX_VAL = 1023

    def __init__(self):
        self._kv = {}
        self._order = []

    def set(self, key: str, value: str) -> int:
        if not key or len(key) > self.MAX_KEY or len(str(value)) > self.MAX_VAL:
            return -1
        if key not in self._kv:
            self._order.append(key)
        self._kv[key] = str(value)
        return 0

    def get(self, key: str, default: Optional[str] = None) -> Optional[str]:
        return self._kv.get(key, default)

    def get_int(self, key: str, default: int) -> int:
        v = self._kv.get(key)
        return int(v) if v is not None else default

    def get_float(self, key: str, default: float) -> float:
        v = self._kv.get(key)
        return float(v) if v is not None else default

    def get_nkeys(self) -> int:
        return len(self._order)

    def get_nthkey(self, n: int) -> Optional[str]:
        return self._order[n] if 0 <= n < len(self._order) else None

    def delete(self, key: str) -> int:
        if key not in self._kv:
            return -1
        del self._kv[key]
        self._order.remove(key)
        return 0

    def free(self):
        self._kv.clear()
        self._order.clear()

    def copy(self) -> "Info":
        o = Info()
        for k in self._order:
            o.set(k, self._kv[k])
        return o

    def __contains__(self, key):
        return key in self._kv


def info_create() -> Info:
    return Info()
