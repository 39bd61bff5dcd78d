#!/bin/bash
# image name / tag of the megatron-deepspeed workload image (built FROM the mxtrain base image)
export IMAGE_NAME=${IMAGE_NAME:-megatron-deepspeed}
export IMAGE_TAG=${IMAGE_TAG:-rocm7.2-gfx950}
