#!/bin/bash
# Round-4 A/B sets k + l in one box session (DEV TOOL)
bash scripts/ab_r4l.sh || exit 1
bash scripts/ab_r4k.sh || exit 1
