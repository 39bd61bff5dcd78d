#!/bin/bash
# image name / tag of the mxtrain runtime image (cf. the reference's per-image set_env.sh)
export IMAGE_NAME=${IMAGE_NAME:-mxtrain}
export IMAGE_TAG=${IMAGE_TAG:-rocm7.2-gfx950}
