"""Katib-compatible Python SDK: ``from katib_amd import sdk as katib``;
``katib.KatibClient``, ``katib.search.double(...)``, ``katib.V1beta1Experiment`` ..."""

from ..api.models import *  # noqa: F401,F403  (V1beta1* models, like kubeflow.katib)
from . import search  # noqa: F401
from .constants import (BASE_IMAGE_MXNET, BASE_IMAGE_PYTORCH, BASE_IMAGE_TENSORFLOW,  # noqa: F401
                        BASE_IMAGE_TENSORFLOW_GPU)
from .katib_client import KatibClient  # noqa: F401
