#!/bin/bash
set -o pipefail
TAG=skd512 bash tools/ab_lib.sh libvcg_w_skd512.so || exit 7
TAG=skd2048 bash tools/ab_lib.sh libvcg_w_skd2048.so || exit 8
