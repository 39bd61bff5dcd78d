#!/bin/bash
# Build the aws-samples-maskrcnn workload image on top of the mxtrain base image (built first if missing),
# push it to $REGISTRY and point the examples that use it at the pushed reference
# (reference: containers/aws-samples-maskrcnn/build_tools/build_and_push.sh, without the ECR specifics).
#   REGISTRY=registry.local:5000 containers/aws-samples-maskrcnn/build_tools/build_and_push.sh [--no-push]
set -e
DIR=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$DIR/../../.." && pwd)
source "$ROOT/containers/mxtrain-rocm/build_tools/set_env.sh"
BASE="$IMAGE_NAME:$IMAGE_TAG"
docker image inspect "$BASE" > /dev/null 2>&1 || \
    docker build -f "$ROOT/containers/mxtrain-rocm/Dockerfile" -t "$BASE" "$ROOT"
source "$DIR/set_env.sh"
REGISTRY=${REGISTRY:?set REGISTRY=<host[:port]/namespace>}
IMAGE="$REGISTRY/$IMAGE_NAME:$IMAGE_TAG"
docker build --build-arg BASE="$BASE" -f "$ROOT/containers/aws-samples-maskrcnn/Dockerfile" -t "$IMAGE_NAME:$IMAGE_TAG" "$ROOT/containers/aws-samples-maskrcnn"
docker tag "$IMAGE_NAME:$IMAGE_TAG" "$IMAGE"
if [ "$1" != "--no-push" ]; then docker push "$IMAGE"; fi
python3 -m mxtrain.tools.images set "$IMAGE" --match "aws-samples-maskrcnn" "$ROOT/examples" "$ROOT/charts/machine-learning"
