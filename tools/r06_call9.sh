#!/bin/bash
# round 6, final build: random differential campaign, the secondary bench
# configs, the N = 2 rehearsal with the new labels
bash tools/gpu_round.sh r06i fuzz sweep dist2
