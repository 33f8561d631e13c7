#!/bin/bash
cd "$(dirname "$0")/.."
for v in "$@"; do timeout -k 5 120 python -u k6lab/probe.py ${v/:/ } || exit 1; done
