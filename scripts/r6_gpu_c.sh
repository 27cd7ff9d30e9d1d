#!/bin/bash
# round 6: the face operator on partitions, agglomerated coarsest level vs per-sweep (detached ranks)
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u scripts/face_strong_probe.py 5 10 1 > $O/r6_face_agg1.txt 2>&1 && \
timeout -k 10 300 python -u scripts/face_strong_probe.py 5 10 0 > $O/r6_face_agg0.txt 2>&1 && \
timeout -k 10 300 python -u scripts/face_strong_probe.py 5 10 1 > $O/r6_face_agg1b.txt 2>&1
