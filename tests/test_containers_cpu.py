"""Container images: the base image plus the four workload images that
mirror the reference's containers/ (megatron-deepspeed, ray-pytorch, tensorpack-maskrcnn,
aws-samples-maskrcnn).  No docker daemon here, so the specs are checked statically:
every module a Dockerfile imports or shims through runpy must import, the shim paths the
charts run must be created by the image that serves them, and every build script parses."""
import glob
import importlib
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOAD_IMAGES = ["megatron-deepspeed", "ray-pytorch", "tensorpack-maskrcnn", "aws-samples-maskrcnn"]


def _dockerfile(name):
    with open(os.path.join(ROOT, "containers", name, "Dockerfile")) as f:
        return f.read()


@pytest.mark.parametrize("name", ["mxtrain-rocm"] + WORKLOAD_IMAGES)
def test_dockerfile_modules_import(name):
    text = _dockerfile(name)
    assert re.search(r"^FROM ", text, re.M)
    mods = set(re.findall(r'run_module\("([\w.]+)"', text))
    for stmt in re.findall(r'python3 -c "import ([\w., ]+)"', text):
        mods |= {m.strip() for m in stmt.split(",")}
    mods |= set(re.findall(r"python3 -m ([\w.]+)", text)) - {"pip", "mxtrain.build"}
    for m in sorted(mods):
        importlib.import_module(m)


@pytest.mark.parametrize("name", WORKLOAD_IMAGES)
def test_workload_images_build_on_base(name):
    text = _dockerfile(name)
    assert "ARG BASE=mxtrain:rocm7.2-gfx950" in text and "FROM ${BASE}" in text
    for script in glob.glob(os.path.join(ROOT, "containers", name, "build_tools", "*.sh")):
        subprocess.check_call(["bash", "-n", script])


def test_chart_script_paths_exist_in_images():
    """The Mask R-CNN charts / reference examples run these paths inside the image."""
    assert "/tensorpack/examples/FasterRCNN/train.py" in _dockerfile("tensorpack-maskrcnn")
    assert "/mask-rcnn-tensorflow/MaskRCNN/train.py" in _dockerfile("aws-samples-maskrcnn")
    assert "/Megatron-DeepSpeed/pretrain_gpt.py" in _dockerfile("megatron-deepspeed")
    for s in glob.glob(os.path.join(ROOT, "containers", "*", "build_tools", "*.sh")) + \
            [os.path.join(ROOT, "build-images.sh")]:
        subprocess.check_call(["bash", "-n", s])
