#!/bin/bash
# snapshot the committed tree into _old/ (git-ignored) and build it, for same-box A/B runs
set -e
cd "$(dirname "$0")/.."
rm -rf _old && mkdir -p _old
git archive HEAD | tar -x -C _old
(cd _old && python -c "import __graft_entry__ as g; g.build()" > /dev/null)
echo "_old/ = $(git rev-parse --short HEAD)"
