# Resource usage of the product render kernel variant (<false, true>) of the current source
make -s -C raytracinginaweekend_amd/csrc resources 2>&1 | awk '/Function Name/ {p = ($0 ~ /ILb0ELb1/)} p && /VGPRs:|Spill|ScratchSize|Occupancy|LDS/ {sub(/.*remark: +/, ""); sub(/ \[-Rpass.*/, ""); printf "%s; ", $0} END {print ""}'
