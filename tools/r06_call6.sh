#!/bin/bash
# round 6: changed GPU tests, then the B4 / B5 A/Bs
bash tools/r06_call1.sh
bash tools/r06_call5.sh
