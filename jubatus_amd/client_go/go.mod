module jubatus_amd

go 1.18

require github.com/ugorji/go/codec v1.2.11
