#!/bin/bash
# Build (and push) every image under containers/ (reference: build-ecr-images.sh, C17).
#   REGISTRY=registry.local:5000 ./build-images.sh
set -e
for s in containers/*/build_tools/build_and_push.sh; do bash "$s" "$@"; done
