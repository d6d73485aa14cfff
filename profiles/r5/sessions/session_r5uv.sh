#!/bin/bash
# r5u + r5v in one box session
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash profiles/r5/sessions/session_r5u.sh || exit 1
bash profiles/r5/sessions/session_r5v.sh || exit 1
