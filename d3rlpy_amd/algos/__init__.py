"""Algorithms on the HIP update engine (reference: d3rlpy/algos/__init__.py).

Only the algorithms on the accelerated hot path are provided.
"""
from .bcq import BCQ
from .cql import CQL, DiscreteCQL
from .dqn import DQN, DoubleDQN
from .sac import SAC
from .td3 import DDPG, TD3
from .td3_plus_bc import TD3PlusBC

__all__ = ["BCQ", "CQL", "DDPG", "DQN", "DiscreteCQL", "DoubleDQN", "SAC", "TD3", "TD3PlusBC", "get_algo"]

ALGO_LIST = {"bcq": BCQ, "cql": CQL, "ddpg": DDPG, "sac": SAC, "td3": TD3, "td3_plus_bc": TD3PlusBC}


DISCRETE_ALGO_LIST = {"cql": DiscreteCQL, "dqn": DQN, "double_dqn": DoubleDQN}


def get_algo(name: str, discrete: bool):
    """algos/__init__.py:66-85 for the algorithms available here."""
    if discrete:
        if name not in DISCRETE_ALGO_LIST:
            raise ValueError(f"discrete {name} is not available on the HIP engine")
        return DISCRETE_ALGO_LIST[name]
    if name not in ALGO_LIST:
        raise ValueError(f"{name} is not available on the HIP engine")
    return ALGO_LIST[name]
