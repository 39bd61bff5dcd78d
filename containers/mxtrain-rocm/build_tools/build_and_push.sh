#!/bin/bash
# Build the mxtrain image, push it to $REGISTRY (any OCI registry), then point every
# example / chart `image:` field at it -- the reference's build_and_push.sh flow
# (ECR describe/create, docker build/tag/push, sed of image: fields)
# without the AWS-specific parts.
#   REGISTRY=registry.local:5000 containers/mxtrain-rocm/build_tools/build_and_push.sh [--no-push]
set -e
DIR=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$DIR/../../.." && pwd)
source "$DIR/set_env.sh"
REGISTRY=${REGISTRY:?set REGISTRY=<host[:port]/namespace>}
IMAGE="$REGISTRY/$IMAGE_NAME:$IMAGE_TAG"
docker build -f "$ROOT/containers/mxtrain-rocm/Dockerfile" -t "$IMAGE_NAME:$IMAGE_TAG" "$ROOT"
docker tag "$IMAGE_NAME:$IMAGE_TAG" "$IMAGE"
if [ "$1" != "--no-push" ]; then docker push "$IMAGE"; fi
python3 -m mxtrain.tools.images set "$IMAGE" "$ROOT/examples" "$ROOT/charts/machine-learning"
