// Common part of the generated Go clients (jenerator -l go).
//
// Reference: jubatus/client/common/{client,datum}.hpp. Transport: net/rpc
// with the msgpack-RPC client codec of github.com/ugorji/go/codec (structs
// travel as arrays, the wire form of every IDL message); every call sends
// the cluster name first.
package common

import (
	"net"
	"net/rpc"

	"github.com/ugorji/go/codec"
)

// Datum = [string_values, num_values, binary_values]
type StringValue struct {
	Key   string
	Value string
}

type NumValue struct {
	Key   string
	Value float64
}

type BinaryValue struct {
	Key   string
	Value []byte
}

type Datum struct {
	StringValues []StringValue
	NumValues    []NumValue
	BinaryValues []BinaryValue
}

func NewDatum() Datum {
	return Datum{[]StringValue{}, []NumValue{}, []BinaryValue{}}
}

func (d *Datum) AddString(key string, value string) {
	d.StringValues = append(d.StringValues, StringValue{key, value})
}

func (d *Datum) AddNumber(key string, value float64) {
	d.NumValues = append(d.NumValues, NumValue{key, value})
}

func (d *Datum) AddBinary(key string, value []byte) {
	d.BinaryValues = append(d.BinaryValues, BinaryValue{key, value})
}

type ClientBase struct {
	client *rpc.Client
	Name   string
}

func Dial(host string, name string) (*ClientBase, error) {
	conn, err := net.Dial("tcp", host)
	if err != nil {
		return nil, err
	}
	mh := new(codec.MsgpackHandle)
	mh.StructToArray = true
	mh.WriteExt = true
	rpcCodec := codec.MsgpackSpecRpc.ClientCodec(conn, mh)
	return &ClientBase{rpc.NewClientWithCodec(rpcCodec), name}, nil
}

// Call sends [name, args...] and decodes the result into *result
func (c *ClientBase) Call(method string, result interface{}, args ...interface{}) error {
	full := append([]interface{}{c.Name}, args...)
	return c.client.Call(method, codec.MsgpackSpecRpcMultiArgs(full), result)
}

func (c *ClientBase) Close() error {
	return c.client.Close()
}

func (c *ClientBase) GetConfig() (string, error) {
	var result string
	err := c.Call("get_config", &result)
	return result, err
}

func (c *ClientBase) Save(id string) (map[string]string, error) {
	var result map[string]string
	err := c.Call("save", &result, id)
	return result, err
}

func (c *ClientBase) Load(id string) (bool, error) {
	var result bool
	err := c.Call("load", &result, id)
	return result, err
}

func (c *ClientBase) GetStatus() (map[string]map[string]string, error) {
	var result map[string]map[string]string
	err := c.Call("get_status", &result)
	return result, err
}

func (c *ClientBase) DoMix() (bool, error) {
	var result bool
	err := c.Call("do_mix", &result)
	return result, err
}

func (c *ClientBase) GetProxyStatus() (map[string]map[string]string, error) {
	var result map[string]map[string]string
	err := c.Call("get_proxy_status", &result)
	return result, err
}
