"""Search-space helpers (reference ``sdk/python/v1beta1/kubeflow/katib/api/search.py:19-64``)."""

from typing import List

from ..api import models


def double(min: float, max: float, step: float = None):
    """Sample a float value uniformly between `min` and `max`."""
    p = models.V1beta1ParameterSpec(parameter_type="double",
                                    feasible_space=models.V1beta1FeasibleSpace(min=str(min), max=str(max)))
    if step is not None:
        p.feasible_space.step = str(step)
    return p


def int(min: int, max: int, step: int = None):  # noqa: A001 - reference name
    """Sample an integer value uniformly between `min` and `max`."""
    p = models.V1beta1ParameterSpec(parameter_type="int",
                                    feasible_space=models.V1beta1FeasibleSpace(min=str(min), max=str(max)))
    if step is not None:
        p.feasible_space.step = str(step)
    return p


def categorical(list: List):  # noqa: A002 - reference name
    """Sample a categorical value from the `list`."""
    return models.V1beta1ParameterSpec(parameter_type="categorical",
                                       feasible_space=models.V1beta1FeasibleSpace(list))
