#!/bin/bash
# image name / tag of the aws-samples-maskrcnn workload image (built FROM the mxtrain base image)
export IMAGE_NAME=${IMAGE_NAME:-aws-samples-maskrcnn}
export IMAGE_TAG=${IMAGE_TAG:-rocm7.2-gfx950}
