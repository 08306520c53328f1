module github.com/westerndigitalcorporation/blb/internal/rsgpu

go 1.21

require github.com/klauspost/reedsolomon v0.0.0-20180704173009-925cb01d6510
