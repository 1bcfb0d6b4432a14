"""The ``State`` interface that mctslib searches over (mctslib/abc/mcts.py:8-30).

Restated here so the facade does not depend on the reference package; mctslib
only duck-types its states, so a BoardV2 from this package drops into
``mctslib.standard.MCTS`` unchanged.
"""
from abc import ABC, abstractmethod
from typing import Any, List


class State(ABC):
    @property
    @abstractmethod
    def legal_actions(self) -> List[Any]:
        raise NotImplementedError

    @abstractmethod
    def apply_action(self, action) -> "State":
        raise NotImplementedError

    @property
    @abstractmethod
    def is_terminal(self) -> bool:
        raise NotImplementedError

    @property
    @abstractmethod
    def reward(self) -> float:
        raise NotImplementedError

    @abstractmethod
    def clone(self):
        raise NotImplementedError
