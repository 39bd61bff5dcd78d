#!/bin/bash
# image name / tag of the ray-pytorch workload image (built FROM the mxtrain base image)
export IMAGE_NAME=${IMAGE_NAME:-ray-pytorch}
export IMAGE_TAG=${IMAGE_TAG:-rocm7.2-gfx950}
