# Common part of the generated Ruby clients (jenerator -l ruby).
#
# Reference: the Ruby client runtime of jubatus-ruby (Jubatus::Common::
# ClientBase / Datum) and jubatus/client/common/{client,datum}.hpp: every
# call sends [cluster name, args...]; the common methods are get_config,
# save, load, get_status, do_mix and get_proxy_status. Transport: the
# msgpack-rpc gem (MessagePack::RPC::Client), the same wire protocol the
# native transport (csrc/native/jb_rpc.cpp) serves.
require 'msgpack/rpc'

module Jubatus
  module Common
    # datum = [string_values, num_values, binary_values]
    class Datum
      attr_reader :string_values, :num_values, :binary_values

      def initialize(values = {})
        @string_values = []
        @num_values = []
        @binary_values = []
        values.each { |k, v| add(k, v) }
      end

      def add(key, value)
        case value
        when String
          if value.encoding == Encoding::BINARY
            @binary_values << [key, value]
          else
            @string_values << [key, value]
          end
        when Integer, Float
          @num_values << [key, value.to_f]
        else
          raise TypeError, "datum value must be a String or a number: #{value.inspect}"
        end
        self
      end

      def to_msgpack(out = '')
        [@string_values, @num_values, @binary_values].to_msgpack(out)
      end

      def self.from_msgpack(v)
        d = new
        v[0].each { |k, s| d.string_values << [k, s] }
        v[1].each { |k, n| d.num_values << [k, n] }
        (v[2] || []).each { |k, b| d.binary_values << [k, b] }
        d
      end
    end

    class ClientBase
      attr_accessor :name

      def initialize(host, port, name, timeout_sec = 10)
        @client = MessagePack::RPC::Client.new(host, port)
        @client.timeout = timeout_sec
        @name = name
      end

      def get_client
        @client
      end

      def close
        @client.close
      end

      def call(method, *args)
        @client.call(method, @name, *args)
      end

      def get_config
        call('get_config')
      end

      def save(id)
        call('save', id)
      end

      def load(id)
        call('load', id)
      end

      def get_status
        call('get_status')
      end

      def do_mix
        call('do_mix')
      end

      def get_proxy_status
        call('get_proxy_status')
      end
    end
  end
end
