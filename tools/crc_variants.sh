#!/bin/bash
# Load-path variants of the standalone CRC kernel (crc32c.hip) for tools/crc_pmc.sh.
set -e
SRCS=crc32c bash "$(dirname "$0")/ect_variants.sh" crc_coal1:"-DBLBRS_CRC_COAL=1" crc_coal0:"-DBLBRS_CRC_COAL=0"
