"""SDK constants (reference ``sdk/python/v1beta1/kubeflow/katib/constants/constants.py:17-58``)."""

import os

DEFAULT_TIMEOUT = 120
KATIB_VERSION = os.environ.get("EXPERIMENT_VERSION", "v1beta1")
KUBEFLOW_GROUP = "kubeflow.org"
EXPERIMENT_KIND = "Experiment"
EXPERIMENT_PLURAL = "experiments"
SUGGESTION_PLURAL = "suggestions"
TRIAL_PLURAL = "trials"
DEFAULT_PRIMARY_CONTAINER_NAME = "training-container"
EXPERIMENT_LABEL = "katib.kubeflow.org/experiment"
CONDITION_STATUS_TRUE = "True"
EXPERIMENT_CONDITION_CREATED = "Created"
EXPERIMENT_CONDITION_RUNNING = "Running"
EXPERIMENT_CONDITION_RESTARTING = "Restarting"
EXPERIMENT_CONDITION_SUCCEEDED = "Succeeded"
EXPERIMENT_CONDITION_FAILED = "Failed"
TRIAL_CONDITION_SUCCEEDED = "Succeeded"
# base images are informational on a node-local scheduler: trials run in the host image
BASE_IMAGE_TENSORFLOW = "docker.io/tensorflow/tensorflow:2.13.0"
BASE_IMAGE_TENSORFLOW_GPU = "docker.io/tensorflow/tensorflow:2.13.0-gpu"
BASE_IMAGE_PYTORCH = "rocm/pytorch:latest"
BASE_IMAGE_MXNET = "docker.io/mxnet/python:1.9.1_native_py3"
DEFAULT_DB_MANAGER_ADDRESS = "katib-db-manager.kubeflow:6789"
