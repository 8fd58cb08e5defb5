set -o pipefail
timeout -k 10 120 python tools/dropin_phases.py && timeout -k 10 120 python tools/dropin_phases.py
