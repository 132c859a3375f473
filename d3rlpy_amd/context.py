"""parallel() / disable_parallel(): the flag stack that makes Device.__deepcopy__
hand out the next GPU id (d3rlpy/context.py:4-22), so sklearn-style cloning
(cross_validate / GridSearchCV with n_jobs) spreads learners over the GPUs."""
from contextlib import contextmanager
from typing import Iterator, List

PARALLEL_FLAG_STACK: List[bool] = [False]


def get_parallel_flag() -> bool:
    return PARALLEL_FLAG_STACK[-1]


@contextmanager
def parallel() -> Iterator[None]:
    PARALLEL_FLAG_STACK.append(True)
    try:
        yield
    finally:
        PARALLEL_FLAG_STACK.pop(-1)


@contextmanager
def disable_parallel() -> Iterator[None]:
    PARALLEL_FLAG_STACK.append(False)
    try:
        yield
    finally:
        PARALLEL_FLAG_STACK.pop(-1)
